"""quantum_amd -- MI355X-native AES-256-GCM packet sealing for quantum's Encryption plugin path.

Layout:
  include/qgcm.h            C ABI (the drop-in boundary; see INTEGRATION.md for the cgo binding)
  quantum_amd/csrc/         gfx950 HIP kernels + the C ABI implementation -> quantum_amd/libqgcm.so
  quantum_amd/crypto.py     crypto.AES / NewAES / ECDH mirror (crypto/aes.go, crypto/ecdh.go)
  quantum_amd/plugin.py     plugin.Plugin / Encryption / Mock / Sorter mirror (plugin/*.go)
  quantum_amd/common.py     common.Payload and constants mirror (common/payload.go, common.go)
  quantum_amd/batch.py      device-resident batch entry points (throughput path)
  quantum_amd/worker.py     worker.Outgoing / Incoming pipeline mirror (worker/outgoing.go, incoming.go)
"""
from . import common, plugin, worker  # noqa: F401
from ._lib import QgcmError, lib  # noqa: F401

__all__ = ["common", "plugin", "worker", "crypto", "batch", "lib", "QgcmError"]


def __getattr__(name):
    if name in ("crypto", "batch"):
        import importlib

        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
