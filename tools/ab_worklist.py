"""Config 3 (bench.extra_config3: 2^20 ragged packets, 1024 keys, device-resident) with the worklist's
counting sort (QGCM_WORKLIST_SORT=count) and the radix sort (the default), alternating in one process;
the first round checks the golden digests.

    python3 tools/ab_worklist.py [rounds]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main() -> None:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    for r in range(rounds):
        for sort in ("count", "radix"):
            os.environ["QGCM_WORKLIST_SORT"] = sort
            out = bench.extra_config3(verify=(r == 0))
            print(json.dumps({"sort": sort, **{k: out.get(k) for k in ("value", "seal_ms", "open_ms", "status_ok",
                                                                      "digest_sealed_ok", "digest_opened_ok")}}),
                  flush=True)
    os.environ.pop("QGCM_WORKLIST_SORT", None)


if __name__ == "__main__":
    main()
