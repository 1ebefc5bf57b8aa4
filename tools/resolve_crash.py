"""Resolve the raw addresses of a glog-style crash report ("@ 0x7f.. (unknown)", "PC: @ 0x7f..") to
library + offset with the /proc/self/maps the crashing process wrote (tools/microbench/pcie.py
PCIE_MAPS), then to symbols with llvm-symbolizer (ROCm's, /opt/rocm/lib/llvm/bin).
Usage: python3 tools/resolve_crash.py <crash log> <maps file>"""
import re
import subprocess
import sys


def load_maps(path):
    out = []
    for ln in open(path):
        parts = ln.split()
        if len(parts) < 6 or not parts[5].startswith("/"):
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        out.append((lo, hi, int(parts[2], 16), parts[5]))
    return out


def main():
    log, maps = sys.argv[1], load_maps(sys.argv[2])
    sym = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"
    for ln in open(log):
        m = re.search(r"@\s+(0x[0-9a-f]+)", ln)
        if not m:
            continue
        a = int(m.group(1), 16)
        hit = next(((lo, hi, off, lib) for lo, hi, off, lib in maps if lo <= a < hi), None)
        if not hit:
            print(f"{m.group(1)}  (not in a file mapping)  | {ln.strip()}")
            continue
        lo, hi, off, lib = hit
        rel = a - lo + off
        try:
            r = subprocess.run([sym, f"--obj={lib}", "--functions=linkage", "--demangle", hex(rel)],
                               capture_output=True, text=True, timeout=60)
            fn = r.stdout.strip().splitlines()[0] if r.stdout.strip() else "?"
        except (OSError, subprocess.SubprocessError):
            fn = "?"
        print(f"{m.group(1)}  {lib}+{hex(rel)}  {fn}")


if __name__ == "__main__":
    main()
