"""A/B the kernel variants in ONE process, interleaved rounds (guide rule 24).  Each variant is a
separate qgcm context (QGCM_VARIANT read at qgcm_create).  Also checks each variant's sealed bytes
against the committed digest of the 4096-packet batch."""
import hashlib, json, os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from quantum_amd import batch
from quantum_amd.crypto import Context, derive_key

variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,3,4".split(","))]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N, L = 1 << 20, 1350
stride = int(os.environ.get("STRIDE", "1408")); OFF = int(os.environ.get("OFF", "60"))
key = derive_key(b"AES256Key-32Characters1234567890", bytes(range(32)))
ctxs = {}
for v in variants:
    os.environ["QGCM_VARIANT"] = str(v)
    c = Context(0, 4); c.set_key(0, key); ctxs[v] = c
dg = json.load(open("tests/golden/batch_digest.json"))[0]
for v, c in ctxs.items():
    n = dg["n"]; stride = dg["stride"]
    a = torch.zeros(n * stride, dtype=torch.uint8, device="cuda"); no = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    batch.fill_uniform(a, stride, n, L, int.from_bytes(bytes([10, 99, 0, 1]), "little"), dg["seed_payload"], no, dg["seed_nonce"])
    batch.seal_uniform(c, a, stride, n, L, 0, no)
    ok = hashlib.sha256(a.cpu().numpy().tobytes()).hexdigest() == dg["sha256_sealed"]
    print(f"variant {v}: digest_ok={ok}", flush=True)
stride = int(os.environ.get("STRIDE", "1408"))
arena_t = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
arena = arena_t[OFF:]
nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
batch.fill_uniform(arena, stride, N, L, 0x0100630a, 0x5EED0001, nonces, 0x5EED0002)
res = {v: ([], []) for v in variants}
for r in range(rounds):
    for v, c in ctxs.items():
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(); batch.seal_uniform(c, arena, stride, N, L, 0, nonces); e[1].record()
        batch.open_uniform(c, arena, stride, N, L + 28, 0); e[2].record(); torch.cuda.synchronize()
        if r > 0:
            res[v][0].append(e[0].elapsed_time(e[1])); res[v][1].append(e[1].elapsed_time(e[2]))
for v in variants:
    s, o = statistics.median(res[v][0]), statistics.median(res[v][1])
    print(f"variant {v}: seal {s:.3f} ms (min {min(res[v][0]):.3f})  open {o:.3f} ms (min {min(res[v][1]):.3f})  "
          f"-> {2*N*L/((s+o)*1e-3)/2**30:.1f} GiB/s", flush=True)
