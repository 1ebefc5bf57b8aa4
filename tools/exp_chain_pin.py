"""Config 5 from host memory (bench.extra_config5: every codec mode) with the chain's snappy workers
pinned one per physical core (QGCM_CHAIN_PIN=1, the default since round 5) or left to the scheduler (0),
alternating in one process, a context per setting (the knob is read at qgcm_create).

    python3 tools/exp_chain_pin.py [rounds] [threads]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main() -> None:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else bench.host_cpus()["share"]
    key = bench.derive_key(bench.SECRET, bench.SALT)
    for r in range(rounds):
        for pin in ("1", "0"):
            os.environ["QGCM_CHAIN_PIN"] = pin
            res = bench.extra_config5(key, threads, reps=3, verify=False)
            print(json.dumps({"pin": int(pin), "round": r, "threads": threads, "value": res["value"],
                              "by_mode": {m: v["value"] for m, v in res["by_codec_mode"].items()},
                              "restored": res["restored"]}), flush=True)
    os.environ.pop("QGCM_CHAIN_PIN", None)


if __name__ == "__main__":
    main()
