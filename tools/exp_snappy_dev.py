"""Device snappy codec rate on device-resident slots (config 5's packets: 2^20 x 1350 B, first half
random, second half a repeated HTTP line, stride 1472): compress, seal, open, uncompress, each timed
by HIP events; the result is checked against the plaintext arena.

    python3 tools/exp_snappy_dev.py [reps] [n]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    key = bench.derive_key(bench.SECRET, bench.SALT)
    for _ in range(2):
        print(json.dumps(bench.extra_config5_resident(key, reps, n)), flush=True)


if __name__ == "__main__":
    main()
