"""A/B whole builds of libqgcm in ONE process (config 2, interleaved rounds).

Each argument is a .so path (e.g. quantum_amd/libqgcm.so and ab/libqgcm_base.so from
tools/build_rev.sh).  Every build seals the same batch; the sealed bytes must agree.
Usage: python tools/ab_libs.py lib1.so lib2.so [...] [--rounds R]
"""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
rounds = 7
if "--rounds" in sys.argv:
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1])
    args = [a for a in args if a != str(rounds)]
N, L = 1 << 20, 1350
stride = 1408
vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
libs = {}
for path in args:
    lib = C.CDLL(os.path.abspath(path))
    lib.qgcm_create.restype = vp
    lib.qgcm_create.argtypes = [C.c_int, u32, C.c_char_p, C.c_size_t]
    lib.qgcm_set_key.argtypes = [vp, u32, C.c_char_p]
    lib.qgcm_derive_key.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p]
    lib.qgcm_seal_uniform.argtypes = [vp, vp, u64, u32, u32, u32, vp, u32, vp, vp]
    lib.qgcm_open_uniform.argtypes = [vp, vp, u64, u32, u32, u32, u32, vp, vp]
    lib.qgcm_fill_uniform.argtypes = [vp, u64, u32, u32, u32, u64, vp, u64, vp]
    err = C.create_string_buffer(120)
    ctx = lib.qgcm_create(0, 4, err, 120)
    assert ctx, err.value
    key = C.create_string_buffer(32)
    secret = b"AES256Key-32Characters1234567890"
    assert lib.qgcm_derive_key(secret, 32, bytes(range(32)), 32, key) == 0
    assert lib.qgcm_set_key(ctx, 0, key.raw) == 0
    libs[path] = (lib, ctx)
alloc = torch.zeros(N * stride + 64, dtype=torch.uint8, device="cuda")
arena = alloc[60:60 + N * stride]
nonces = torch.zeros(12 * N, dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
first = next(iter(libs.values()))[0]
first.qgcm_fill_uniform(arena.data_ptr(), stride, N, L, 0x0100630a, 0x5EED0001, nonces.data_ptr(), 0x5EED0002,
                        stream)
plain = arena.clone()
ref = None
for path, (lib, ctx) in libs.items():
    arena.copy_(plain)
    assert lib.qgcm_seal_uniform(ctx, arena.data_ptr(), stride, N, L, 0, nonces.data_ptr(), 4, None, stream) == 0
    if ref is None:
        ref = arena.clone()
    same = bool(torch.equal(arena, ref))
    assert lib.qgcm_open_uniform(ctx, arena.data_ptr(), stride, N, L + 28, 0, 4, None, stream) == 0
    rt = bool(torch.equal(arena.view(N, stride)[:, :4 + L], plain.view(N, stride)[:, :4 + L]))
    print(f"{path}: sealed bytes same as first: {same}; round trip: {rt}", flush=True)
res = {p: ([], []) for p in libs}
for r in range(rounds + 1):
    for path, (lib, ctx) in libs.items():
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        lib.qgcm_seal_uniform(ctx, arena.data_ptr(), stride, N, L, 0, nonces.data_ptr(), 4, None, stream)
        e[1].record()
        lib.qgcm_open_uniform(ctx, arena.data_ptr(), stride, N, L + 28, 0, 4, None, stream)
        e[2].record()
        torch.cuda.synchronize()
        if r > 0:
            res[path][0].append(e[0].elapsed_time(e[1]))
            res[path][1].append(e[1].elapsed_time(e[2]))
for path in libs:
    s, o = statistics.median(res[path][0]), statistics.median(res[path][1])
    print(f"{path}: seal {s:.3f} ms  open {o:.3f} ms  -> {2 * N * L / ((s + o) * 1e-3) / 2**30:.1f} GiB/s", flush=True)
