"""Is the device snappy encoder occupancy-bound?    The four-packets-per-wave
encoder holds 7 waves per CU, capped by 5.5 KiB of LDS per packet (hash table + staged input).  Before
moving the input out of LDS (which puts a vector-memory load on every miss probe's critical path),
this measures how the encoder's time scales with the waves per CU it is given: QGCM_SNAPPY_PER_CU caps
the resident codec waves per CU (read at qgcm_create, so a context per setting), alternating in one
process on config 5's device-resident packets (bench.extra_config5_resident: compress, seal, open,
uncompress by HIP events; the first round checks every setting's sealed arena against
tests/golden/config5_digest.json, every round the restored plaintext).

    python3 tools/exp_snappy_occupancy.py [reps] [rounds]      (SNAP_PER_CU="7,6,5,4,3")
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
        for per_cu in os.environ.get("SNAP_PER_CU", "7,6,5,4,3").split(","):
            os.environ["QGCM_SNAPPY_PER_CU"] = per_cu
            res = bench.extra_config5_resident(key, reps, verify=(r == 0))
            print(json.dumps({"waves_per_cu_cap": int(per_cu), "round": r,
                              **{k: res[k] for k in ("compress_ms", "seal_ms", "open_ms", "uncompress_ms",
                                                     "compress_GBps", "value", "status_ok_and_restored",
                                                     "sealed_digest_ok")}}), flush=True)
    os.environ.pop("QGCM_SNAPPY_PER_CU", None)


if __name__ == "__main__":
    main()
