"""Device snappy codec rate on device-resident slots (config 5's packets: 2^20 x 1350 B, first half
random, second half a repeated HTTP line, stride 1472): compress, seal, open, uncompress, each timed
by HIP events; the sealed arena is checked against tests/golden/config5_digest.json and the result
against the plaintext arena (bench.extra_config5_resident).  The encoders alternate in one process,
`rounds` times each: QGCM_SNAPPY_GROUP=1, four packets per wave in both directions (the default),
and 0, one wave per packet (SNAP_GROUPS="1,2" compares other settings, e.g. a temporary variant wired to 2 for an A/B).

    python3 tools/exp_snappy_dev.py [reps] [rounds]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    key = bench.derive_key(bench.SECRET, bench.SALT)
    for r in range(rounds):
        for grp in os.environ.get("SNAP_GROUPS", "1,0").split(","):
            os.environ["QGCM_SNAPPY_GROUP"] = grp
            res = bench.extra_config5_resident(key, reps, verify=(r == 0))
            print(json.dumps({"snappy_group": int(grp), **res}), flush=True)
    os.environ.pop("QGCM_SNAPPY_GROUP", None)


if __name__ == "__main__":
    main()
