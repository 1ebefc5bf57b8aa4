"""One PCIe-inclusive bench leg in this process (for tracing it under rocprofv3):
    python3 tools/run_leg.py e2e|config3_host [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402

leg = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
if leg == "e2e":
    out = bench.extra_e2e(bench.derive_key(bench.SECRET, bench.SALT), reps=reps)
elif leg == "config3_host":
    out = bench.extra_config3_host(reps=reps, verify=False)
else:
    raise SystemExit("unknown leg " + leg)
print(json.dumps(out), flush=True)
