"""Device-resident packet batches: the throughput path for workers that hand over whole batches
(worker/outgoing.go:55-93 and worker/incoming.go:54-92 loop over packets).

Slots are common.Payload.Raw buffers laid end to end in one HBM arena (include/qgcm.h).  Torch
is used only as the device allocator and for stream handles; the work is done by libqgcm.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .crypto import Context

AAD_LEN = 4  # the Payload IP header is the additional data (plugin/encryption.go:22,31)


def _stream_handle(stream: torch.cuda.Stream | None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else int(t.data_ptr())


def slot_stride(max_len: int, align: int = 16) -> int:
    """Smallest multiple of `align` holding [aad 4][payload][tag 16][nonce 12]."""
    return (4 + max_len + _lib.OVERHEAD + align - 1) // align * align


def seal_uniform(ctx: Context, arena: torch.Tensor, stride: int, n: int, length: int, key_idx: int,
                 nonces: torch.Tensor | None = None, aad_len: int = AAD_LEN, status: torch.Tensor | None = None,
                 stream: torch.cuda.Stream | None = None) -> None:
    _lib.check(_lib.lib().qgcm_seal_uniform(ctx.handle, _ptr(arena), stride, n, length, key_idx, _ptr(nonces),
                                            aad_len, _ptr(status), _stream_handle(stream)), "qgcm_seal_uniform")


def open_uniform(ctx: Context, arena: torch.Tensor, stride: int, n: int, sealed_len: int, key_idx: int,
                 aad_len: int = AAD_LEN, status: torch.Tensor | None = None,
                 stream: torch.cuda.Stream | None = None) -> None:
    _lib.check(_lib.lib().qgcm_open_uniform(ctx.handle, _ptr(arena), stride, n, sealed_len, key_idx, aad_len,
                                            _ptr(status), _stream_handle(stream)), "qgcm_open_uniform")


def make_descs(offsets, lengths, keys, device) -> torch.Tensor:
    """Pack qgcm_desc records ({u64 offset, u32 len, u32 key_idx}) into a device uint8 tensor."""
    def col(x) -> torch.Tensor:
        if isinstance(x, np.ndarray):  # unsigned numpy arrays (uint64 offsets) go through int64
            x = x.astype(np.int64)
        return torch.as_tensor(x, dtype=torch.int64).reshape(-1, 1)

    off, ln, ky = col(offsets), col(lengths), col(keys)
    words = torch.cat([off & 0xFFFFFFFF, off >> 32, ln, ky], dim=1).to(torch.int64)
    words = torch.where(words >= 2**31, words - 2**32, words).to(torch.int32)
    return words.contiguous().view(torch.uint8).reshape(-1).to(device)


def seal_batch(ctx: Context, arena: torch.Tensor, descs: torch.Tensor, n: int, nonces: torch.Tensor | None = None,
               aad_len: int = AAD_LEN, status: torch.Tensor | None = None,
               stream: torch.cuda.Stream | None = None) -> None:
    _lib.check(_lib.lib().qgcm_seal_batch(ctx.handle, _ptr(arena), _ptr(descs), n, _ptr(nonces), aad_len,
                                          _ptr(status), _stream_handle(stream)), "qgcm_seal_batch")


def open_batch(ctx: Context, arena: torch.Tensor, descs: torch.Tensor, n: int, aad_len: int = AAD_LEN,
               status: torch.Tensor | None = None, stream: torch.cuda.Stream | None = None) -> None:
    _lib.check(_lib.lib().qgcm_open_batch(ctx.handle, _ptr(arena), _ptr(descs), n, aad_len, _ptr(status),
                                          _stream_handle(stream)), "qgcm_open_batch")


def fill_uniform(arena: torch.Tensor, stride: int, n: int, length: int, aad_word: int, seed_payload: int,
                 nonces: torch.Tensor | None, seed_nonce: int, stream: torch.cuda.Stream | None = None) -> None:
    """Synthetic slots: payload = splitmix64(seed_payload) stream bytes [i*L, (i+1)*L)."""
    _lib.check(_lib.lib().qgcm_fill_uniform(_ptr(arena), stride, n, length, aad_word, seed_payload, _ptr(nonces),
                                            seed_nonce, _stream_handle(stream)), "qgcm_fill_uniform")


def snappy_compress(ctx: Context, arena: torch.Tensor, stride: int, n: int, lens: torch.Tensor, max_len: int,
                    limit: int, status: torch.Tensor | None = None, descs_out: torch.Tensor | None = None,
                    key_idx: int = 0, stream: torch.cuda.Stream | None = None) -> None:
    """Device snappy Encode of each slot's packet in place (compression.go Outgoing); `lens` a device
    int32/uint32 tensor, updated to the compressed lengths; `descs_out` (16 n bytes) receives the seal
    descriptors of the compressed packets."""
    _lib.check(_lib.lib().qgcm_snappy_compress_batch(ctx.handle, _ptr(arena), stride, n, _ptr(lens), max_len, limit,
                                                     _ptr(status), _ptr(descs_out), key_idx, _stream_handle(stream)),
               "qgcm_snappy_compress_batch")


def snappy_uncompress(ctx: Context, arena: torch.Tensor, stride: int, n: int, lens: torch.Tensor, max_len: int,
                      cap: int, status: torch.Tensor | None = None, stream: torch.cuda.Stream | None = None) -> None:
    """Device snappy Decode of each slot's packet in place (compression.go Incoming)."""
    _lib.check(_lib.lib().qgcm_snappy_uncompress_batch(ctx.handle, _ptr(arena), stride, n, _ptr(lens), max_len, cap,
                                                       _ptr(status), _stream_handle(stream)),
               "qgcm_snappy_uncompress_batch")


def host_ptr(buf: bytearray) -> tuple[int, object]:
    arr = (C.c_uint8 * len(buf)).from_buffer(buf)
    return C.addressof(arr), arr


def compress_seal_host(ctx: Context, arena_ptr: int, stride: int, n: int, lens, key_idx: int, nonces_ptr: int | None,
                       aad_len: int = AAD_LEN, threads: int = 16, status_ptr: int | None = None) -> int:
    """Outgoing plugin chain on host slots (main.go:50-51 order): snappy-compress then seal, pipelined
    with the device.  `lens` is a numpy uint32 array, updated in place to the sealed lengths.
    Returns the number of packets that failed (status 0)."""
    return _lib.check(_lib.lib().qgcm_compress_seal_host(ctx.handle, arena_ptr, stride, n, lens.ctypes.data, key_idx,
                                                         nonces_ptr, aad_len, threads, status_ptr),
                      "qgcm_compress_seal_host")


def chain_codec(ctx: Context, mode: int = -1) -> int:
    """Where the chained calls run the snappy codec (0 host, 1 split, 2 device); returns the previous mode."""
    return _lib.check(_lib.lib().qgcm_chain_codec(ctx.handle, mode), "qgcm_chain_codec")


def open_uncompress_host(ctx: Context, arena_ptr: int, stride: int, n: int, lens, key_idx: int,
                         aad_len: int = AAD_LEN, threads: int = 16, status_ptr: int | None = None) -> int:
    """Incoming plugin chain on host slots: open then snappy-uncompress; `lens` updated in place."""
    return _lib.check(_lib.lib().qgcm_open_uncompress_host(ctx.handle, arena_ptr, stride, n, lens.ctypes.data, key_idx,
                                                           aad_len, threads, status_ptr),
                      "qgcm_open_uncompress_host")
