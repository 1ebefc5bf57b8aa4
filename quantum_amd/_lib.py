"""ctypes binding of libqgcm.so (include/qgcm.h).

The library is the product: every packet is sealed/opened by the gfx950 kernels inside it.
There is no Python or CPU fallback -- if the shared object is missing or no gfx950 device is
present, loading/creating a context raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libqgcm.so")
# tools' A/B runs load another build of the same ABI in its place (never set by the product or the tests)
if os.environ.get("QGCM_AB_LIB"):
    LIB_PATH = os.path.abspath(os.environ["QGCM_AB_LIB"])

# Every symbol include/qgcm.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "qgcm_create", "qgcm_destroy", "qgcm_strerror", "qgcm_version", "qgcm_device_count",
    "qgcm_derive_key", "qgcm_derive_keys", "qgcm_set_key", "qgcm_set_keys", "qgcm_clear_keys",
    "qgcm_x25519_base", "qgcm_x25519",
    "qgcm_seal_batch", "qgcm_open_batch", "qgcm_seal_uniform", "qgcm_open_uniform",
    "qgcm_seal_one", "qgcm_open_one", "qgcm_seal_host", "qgcm_open_host",
    "qgcm_random_nonces", "qgcm_fill_uniform", "qgcm_host_alloc", "qgcm_host_free",
    "qgcm_stream_copy",
    "qgcm_snappy_max_compressed_length", "qgcm_snappy_compress", "qgcm_snappy_uncompressed_length",
    "qgcm_snappy_uncompress", "qgcm_snappy_compress_slots", "qgcm_snappy_uncompress_slots",
    "qgcm_snappy_compress_slots_limit", "qgcm_compress_seal_host", "qgcm_open_uncompress_host",
    "qgcm_snappy_compress_batch", "qgcm_snappy_uncompress_batch", "qgcm_chain_codec",
    "qgcm_udp_socket", "qgcm_udp_queue", "qgcm_udp_port", "qgcm_udp_close", "qgcm_udp_recv_slots",
    "qgcm_udp_send_slots",
    "qgcm_tun_open", "qgcm_tun_up", "qgcm_tun_read_slots", "qgcm_tun_write_slots", "qgcm_tun_close",
    "qgcm_group_create", "qgcm_group_destroy", "qgcm_group_size", "qgcm_group_ctx", "qgcm_group_shard",
    "qgcm_group_set_keys", "qgcm_group_clear_keys", "qgcm_group_seal_host", "qgcm_group_open_host", "qgcm_group_member_cpus",
    "qgcm_group_last_zerocopy", "qgcm_group_last_path", "qgcm_group_order", "qgcm_launch_counts", "qgcm_resident_stop", "qgcm_resident_stats",
)

QGCM_OK = 0
QGCM_E_ARG = -1
QGCM_E_HIP = -2
QGCM_E_KEY = -3
QGCM_E_AUTH = -4
QGCM_E_NOMEM = -5
OVERHEAD = 28
ERRLEN = 120


class QgcmError(RuntimeError):
    pass


class Desc(C.Structure):
    """qgcm_desc: {offset u64, len u32, key_idx u32} -- 16 bytes."""

    _fields_ = [("offset", C.c_uint64), ("len", C.c_uint32), ("key_idx", C.c_uint32)]


_lib: C.CDLL | None = None


def _bind(L: C.CDLL) -> None:
    vp, u8p, sz, u32, u64, i32, lng = C.c_void_p, C.c_char_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int, C.c_long
    L.qgcm_create.argtypes = [i32, u32, C.c_char_p, i32]
    L.qgcm_create.restype = vp
    L.qgcm_destroy.argtypes = [vp]
    L.qgcm_destroy.restype = None
    L.qgcm_strerror.argtypes = [i32]
    L.qgcm_strerror.restype = C.c_char_p
    L.qgcm_version.restype = C.c_char_p
    L.qgcm_device_count.argtypes = []
    L.qgcm_device_count.restype = i32
    L.qgcm_derive_key.argtypes = [u8p, sz, u8p, sz, u8p]
    L.qgcm_derive_keys.argtypes = [u8p, u8p, u32, u8p]
    L.qgcm_set_key.argtypes = [vp, u32, u8p]
    L.qgcm_set_keys.argtypes = [vp, u32, u32, u8p]
    if hasattr(L, "qgcm_clear_keys"):
        L.qgcm_clear_keys.argtypes = [vp, u32, u32]
    L.qgcm_x25519_base.argtypes = [u8p, u8p]
    L.qgcm_x25519.argtypes = [u8p, u8p, u8p]
    L.qgcm_seal_batch.argtypes = [vp, vp, vp, u32, vp, u32, vp, vp]
    L.qgcm_open_batch.argtypes = [vp, vp, vp, u32, u32, vp, vp]
    L.qgcm_seal_uniform.argtypes = [vp, vp, u64, u32, u32, u32, vp, u32, vp, vp]
    L.qgcm_open_uniform.argtypes = [vp, vp, u64, u32, u32, u32, u32, vp, vp]
    L.qgcm_seal_one.argtypes = [vp, u32, vp, lng, vp, u32, vp]
    L.qgcm_seal_one.restype = lng
    L.qgcm_open_one.argtypes = [vp, u32, vp, lng, vp, u32]
    L.qgcm_open_one.restype = lng
    L.qgcm_seal_host.argtypes = [vp, vp, u64, u32, u32, u32, vp, u32, vp]
    L.qgcm_open_host.argtypes = [vp, vp, u64, u32, u32, u32, u32, vp]
    L.qgcm_random_nonces.argtypes = [vp, u32]
    L.qgcm_host_alloc.argtypes = [C.c_size_t]
    L.qgcm_host_alloc.restype = vp
    L.qgcm_host_free.argtypes = [vp]
    L.qgcm_host_free.restype = None
    L.qgcm_stream_copy.argtypes = [vp, vp, vp, u64, vp]
    if hasattr(L, "qgcm_launch_counts"):
        L.qgcm_launch_counts.argtypes = [vp, vp, i32]
    if hasattr(L, "qgcm_resident_stop"):
        L.qgcm_resident_stop.argtypes = [vp]
        L.qgcm_resident_stats.argtypes = [vp, vp, i32]
    sz = C.c_size_t
    L.qgcm_snappy_max_compressed_length.argtypes = [sz]
    L.qgcm_snappy_max_compressed_length.restype = sz
    L.qgcm_snappy_compress.argtypes = [vp, sz, vp, sz]
    L.qgcm_snappy_compress.restype = lng
    L.qgcm_snappy_uncompressed_length.argtypes = [vp, sz]
    L.qgcm_snappy_uncompressed_length.restype = lng
    L.qgcm_snappy_uncompress.argtypes = [vp, sz, vp, sz]
    L.qgcm_snappy_uncompress.restype = lng
    L.qgcm_snappy_compress_slots.argtypes = [vp, u64, u32, vp, C.c_int]
    L.qgcm_snappy_uncompress_slots.argtypes = [vp, u64, u32, vp, vp, C.c_int]
    L.qgcm_fill_uniform.argtypes = [vp, u64, u32, u32, u32, u64, vp, u64, vp]
    L.qgcm_snappy_compress_slots_limit.argtypes = [vp, u64, u32, vp, u64, vp, C.c_int]
    L.qgcm_snappy_compress_batch.argtypes = [vp, vp, u64, u32, vp, u32, u32, vp, vp, u32, vp]
    L.qgcm_snappy_uncompress_batch.argtypes = [vp, vp, u64, u32, vp, u32, u32, vp, vp]
    L.qgcm_chain_codec.argtypes = [vp, i32]
    L.qgcm_compress_seal_host.argtypes = [vp, vp, u64, u32, vp, u32, vp, u32, C.c_int, vp]
    L.qgcm_open_uncompress_host.argtypes = [vp, vp, u64, u32, vp, u32, u32, C.c_int, vp]
    L.qgcm_udp_socket.argtypes = [C.c_char_p, C.c_int, C.c_int]
    L.qgcm_udp_queue.argtypes = [C.c_char_p, C.c_int, C.c_int]
    L.qgcm_udp_port.argtypes = [C.c_int]
    L.qgcm_udp_close.argtypes = [C.c_int]
    L.qgcm_udp_recv_slots.argtypes = [C.c_int, vp, u64, u32, vp, C.c_int]
    L.qgcm_udp_send_slots.argtypes = [C.c_int, vp, u64, u32, vp, C.c_char_p, C.c_int]
    if hasattr(L, "qgcm_group_create"):  # (older builds loaded by the A/B tools lack the group calls)
        L.qgcm_group_create.argtypes = [vp, i32, u32, C.c_char_p, i32]
        L.qgcm_group_create.restype = vp
        L.qgcm_group_destroy.argtypes = [vp]
        L.qgcm_group_destroy.restype = None
        L.qgcm_group_size.argtypes = [vp]
        L.qgcm_group_ctx.argtypes = [vp, i32]
        L.qgcm_group_ctx.restype = vp
        L.qgcm_group_shard.argtypes = [vp, u32]
        L.qgcm_group_set_keys.argtypes = [vp, u32, u32, u8p]
        if hasattr(L, "qgcm_group_clear_keys"):
            L.qgcm_group_clear_keys.argtypes = [vp, u32, u32]
        L.qgcm_group_seal_host.argtypes = [vp, vp, vp, u32, vp, u32, vp]
        L.qgcm_group_open_host.argtypes = [vp, vp, vp, u32, u32, vp]
        if hasattr(L, "qgcm_group_member_cpus"):
            L.qgcm_group_member_cpus.argtypes = [vp, i32]
        if hasattr(L, "qgcm_group_last_zerocopy"):
            L.qgcm_group_last_zerocopy.argtypes = [vp]
        if hasattr(L, "qgcm_group_last_path"):
            L.qgcm_group_last_path.argtypes = [vp, i32]
            L.qgcm_group_order.argtypes = [vp, vp, u32, vp, vp]
    if hasattr(L, "qgcm_tun_open"):  # (older builds loaded by the A/B tools lack the TUN calls)
        L.qgcm_tun_open.argtypes = [C.c_char_p, C.c_int, vp, C.c_char_p, sz]
        L.qgcm_tun_up.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
        L.qgcm_tun_read_slots.argtypes = [C.c_int, vp, u64, u32, vp, C.c_int]
        L.qgcm_tun_write_slots.argtypes = [C.c_int, vp, u64, u32, vp]
        L.qgcm_tun_close.argtypes = [C.c_int]


def lib() -> C.CDLL:
    """Load libqgcm.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QgcmError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        # Share torch's HIP runtime (same SONAME libamdhip64.so.7) when torch is present: import it first.
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is plumbing only
            pass
        L = C.CDLL(LIB_PATH)
        _bind(L)
        _lib = L
    return _lib


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise QgcmError(f"{what}: {lib().qgcm_strerror(rc).decode()} ({rc})")
    return rc
