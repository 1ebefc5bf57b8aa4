"""Runs only the config-5 chain (tools/bench_configs.py config5) -- a target for rocprofv3 traces."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import bench_configs  # noqa: E402

print(json.dumps(bench_configs.config5(reps=1)), flush=True)
