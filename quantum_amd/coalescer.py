"""Cross-thread coalescer over libqgcm (qgcm_coalescer_*).

quantum's 2 x NumWorkers goroutines each call plugin.Apply once per packet (worker/outgoing.go:55-93,
worker/incoming.go:54-92).  A Coalescer keeps that per-packet, blocking Encrypt/Decrypt contract
(crypto/aes.go:41-62) while concurrent callers' packets share one device batch, flushed at
`max_batch` packets or after `max_wait_us`.  Bind it to an AES with `crypto.AES(..., coalescer=c)`
(or `aes.coalescer = c`); ctypes releases the GIL, so Python threads really overlap.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from .common import MaxPacketLength


class Coalescer:
    def __init__(self, ctx, max_batch: int = 4096, max_wait_us: int = 200, max_packet: int = MaxPacketLength,
                 aad_len: int = 4):
        err = C.create_string_buffer(_lib.ERRLEN)
        h = _lib.lib().qgcm_coalescer_create(ctx.handle, max_batch, max_wait_us, max_packet, aad_len, err,
                                             _lib.ERRLEN)
        if not h:
            raise RuntimeError(err.value.decode(errors="replace"))
        self.ctx = ctx
        self.handle = h
        self.max_packet = max_packet

    def close(self) -> None:
        if self.handle:
            _lib.lib().qgcm_coalescer_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
