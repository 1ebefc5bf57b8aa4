"""Config 2 from pinned host memory (bench.extra_e2e: qgcm_seal_host / qgcm_open_host, PCIe included)
with two builds of libqgcm, alternating, each in its own process (QGCM_AB_LIB selects the build).

    python3 tools/exp_e2e_ab.py <lib_a.so> <lib_b.so> [rounds]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = ("import sys, json; sys.path.insert(0, %r); import bench; "
         "print(json.dumps(bench.extra_e2e(bench.derive_key(bench.SECRET, bench.SALT))))" % ROOT)


def main() -> None:
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    for _ in range(rounds):
        for lib in libs:
            env = dict(os.environ, QGCM_AB_LIB=os.path.abspath(lib))
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(json.dumps({"lib": lib, "error": r.stderr[-400:]}), flush=True)
                sys.exit(1)
            print(json.dumps({"lib": lib, **json.loads(r.stdout.strip().splitlines()[-1])}), flush=True)


if __name__ == "__main__":
    main()
