#!/bin/bash
# Builds libqgcm.so variants that differ only in the worklist's rocprim Onesweep configuration
# (quantum_amd/csrc/worklist.hip SortConfig), as absort/libqgcm_s<i>.so, for an in-process A/B on the
# config-3 workload: python3 tools/ab_libs_desc.py absort/*.so.  A stable LSD radix sort gives the same
# order whatever its digit width or tile size, so every variant must seal identical bytes (the A/B
# script checks it).  absort/ is git-ignored but travels to the GPU box.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/absort"
V=(
  "rocprim::default_config"
  "rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 8>, rocprim::kernel_config<256, 8>, 8, rocprim::block_radix_rank_algorithm::match>"
  "rocprim::radix_sort_onesweep_config<rocprim::kernel_config<512, 8>, rocprim::kernel_config<512, 8>, 8, rocprim::block_radix_rank_algorithm::match>"
)
for i in "${!V[@]}"; do
  [ -f "$ROOT/absort/libqgcm_s$i.so" ] && continue
  TMP=$(mktemp -d /tmp/qgcm_sort_XXXX)
  mkdir -p "$TMP/quantum_amd" "$TMP/include"
  cp -r "$ROOT/quantum_amd/csrc" "$TMP/quantum_amd/csrc"
  cp "$ROOT"/include/*.h* "$TMP/include/"
  rm -rf "$TMP/quantum_amd/csrc/_obj"
  python3 - "$TMP/quantum_amd/csrc/worklist.hip" "${V[$i]}" <<'PY'
import sys
p, cfg = sys.argv[1], sys.argv[2]
s = open(p).read()
a = "rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,\n                                              rocprim::default_config, 0>"
assert a in s
open(p, "w").write(s.replace(a, "rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,\n " + cfg + ", 0>"))
PY
  make -s -C "$TMP/quantum_amd/csrc" -j8 OUT="$TMP" >/dev/null
  cp "$TMP/libqgcm.so" "$ROOT/absort/libqgcm_s$i.so"
  rm -rf "$TMP"
  echo "absort/libqgcm_s$i.so: ${V[$i]}"
done
