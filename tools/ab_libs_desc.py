"""A/B whole builds of libqgcm on the config-3 workload (descriptor batches, 1024 keys, lengths
U{64..9000}) in ONE process, interleaved rounds.  Every build seals the same batch; the sealed bytes
must agree.  Usage: python tools/ab_libs_desc.py lib1.so lib2.so [...] [--rounds R]; AB_KEYS=k draws the
key indices from the first k keys (default 1024), AB_LEN=L gives every packet length L.
"""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from quantum_amd import _lib, batch  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
rounds = 5
if "--rounds" in sys.argv:
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1])
    args = [a for a in args if a != str(rounds)]
N, NK = 1 << 20, 1024
rng = np.random.default_rng(0x5EED0003)
keys = rng.bytes(32 * NK)
libs = {}
for path in args:
    L = C.CDLL(os.path.abspath(path))
    _lib._bind(L)
    err = C.create_string_buffer(_lib.ERRLEN)
    ctx = L.qgcm_create(0, NK, err, _lib.ERRLEN)
    assert ctx, err.value
    assert L.qgcm_set_keys(ctx, 0, NK, keys) == 0
    libs[path] = (L, ctx)

lens = rng.integers(64, 9001, size=N, dtype=np.int64)
kidx = rng.integers(0, int(os.environ.get("AB_KEYS", NK)), size=N, dtype=np.int64)
if int(os.environ.get("AB_LEN", 0)):
    lens[:] = int(os.environ["AB_LEN"])
slot = (4 + lens + 28 + 3) & ~3
offs = np.zeros(N, dtype=np.int64)
offs[1:] = np.cumsum(slot)[:-1]
total = int(offs[-1] + slot[-1])
plain = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device="cuda")
arena = plain.clone()
nonces = torch.randint(0, 256, (12 * N,), dtype=torch.uint8, device="cuda")
status = torch.zeros(N, dtype=torch.uint8, device="cuda")
d_seal = batch.make_descs(offs, lens, kidx, "cuda")
d_open = batch.make_descs(offs, lens + 28, kidx, "cuda")
stream = torch.cuda.current_stream().cuda_stream


def seal(L, ctx):
    assert L.qgcm_seal_batch(ctx, arena.data_ptr(), d_seal.data_ptr(), N, nonces.data_ptr(), 4, status.data_ptr(),
                             stream) == 0


def open_(L, ctx):
    assert L.qgcm_open_batch(ctx, arena.data_ptr(), d_open.data_ptr(), N, 4, status.data_ptr(), stream) == 0


ref = ref_open = None
for path, (L, ctx) in libs.items():
    arena.copy_(plain)
    seal(L, ctx)
    ok = int(status.sum()) == N
    if ref is None:
        ref = arena.clone()
    same = bool(torch.equal(arena, ref))
    open_(L, ctx)
    if ref_open is None:
        ref_open = arena.clone()
    rt = int(status.sum()) == N and bool(torch.equal(arena[:64], plain[:64])) and bool(torch.equal(arena, ref_open))
    print(f"{path}: status_ok={ok} sealed bytes same as first: {same}; round trip (whole arena as first): {rt}",
          flush=True)
    assert ok and same and rt, f"{path} differs from {next(iter(libs))}"
payload = int(lens.sum())
res = {p: ([], []) for p in libs}
for r in range(rounds + 1):
    for path, (L, ctx) in libs.items():
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        seal(L, ctx)
        e[1].record()
        open_(L, ctx)
        e[2].record()
        torch.cuda.synchronize()
        if r > 0:
            res[path][0].append(e[0].elapsed_time(e[1]))
            res[path][1].append(e[1].elapsed_time(e[2]))
for path in libs:
    s, o = statistics.median(res[path][0]), statistics.median(res[path][1])
    print(f"{path}: seal {s:.3f} ms  open {o:.3f} ms  -> {2 * payload / ((s + o) * 1e-3) / 2**30:.1f} GiB/s",
          flush=True)
