"""Device snappy codec rate on device-resident slots (config 5's packets: 2^20 x 1350 B, first half
random, second half a repeated HTTP line, stride 1472): compress, seal, open, uncompress, each timed
by HIP events; the sealed arena is checked against tests/golden/config5_digest.json and the result
against the plaintext arena (bench.extra_config5_resident).  Encoder / decoder pairs alternate in one
process, `rounds` times each.  Encoders (QGCM_SNAPPY_GROUP): 3 four packets per wave, pipelined miss
probes, output straight into the slot (the default); 2 the same with the output staged in LDS; 1 not
pipelined; 0 one wave per packet.  Decoders (QGCM_SNAPPY_DEC_GROUP): 1 four packets per wave (the
default), 0 one wave per packet.  The third field sets QGCM_SNAPPY_PREFETCH (the group kernels load
the next packets while coding the current ones; default 1).

    python3 tools/exp_snappy_dev.py [reps] [rounds] [enc:dec:pf,...]   (default 5 2 3:1:1,3:0:1,3:1:0)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    pairs = [(p.split(":") + ["1"])[:3] for p in (sys.argv[3] if len(sys.argv) > 3 else "3:1:1,3:0:1,3:1:0").split(",")]
    key = bench.derive_key(bench.SECRET, bench.SALT)
    for r in range(rounds):
        for enc, dec, pf in pairs:
            os.environ["QGCM_SNAPPY_GROUP"] = enc
            os.environ["QGCM_SNAPPY_DEC_GROUP"] = dec
            os.environ["QGCM_SNAPPY_PREFETCH"] = pf
            res = bench.extra_config5_resident(key, reps, verify=(r == 0))
            print(json.dumps({"snappy_group": int(enc), "snappy_dec_group": int(dec), "prefetch": int(pf), **res}),
                  flush=True)
    for k in ("QGCM_SNAPPY_GROUP", "QGCM_SNAPPY_DEC_GROUP", "QGCM_SNAPPY_PREFETCH"):
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
