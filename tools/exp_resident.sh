#!/bin/bash
# Resident per-packet kernel experiments (tools/bin/per_packet_bench): thread counts, next to a bulk
# host batch, worker count and spinner cap, payload sizes.
set -u
OUT=gpurun_out/${1:-exp_res}
mkdir -p $OUT
run() {  # label, env..., then -- threads payload bulk mode
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  echo "== $label ${envs[*]} $*" >> $OUT/sweep.txt
  env "${envs[@]}" timeout -k 10 60 tools/bin/per_packet_bench "$1" "$2" 1.5 "$3" "$4" >> $OUT/sweep.txt 2>&1
  local rc=$?
  if [ $rc -ge 124 ]; then echo "stop rc=$rc" >> $OUT/sweep.txt; exit $rc; fi
}
for t in 1 4 16 64 256; do
  run t$t X=1 -- $t 1350 0 resident
done
run bulk16 X=1 -- 16 1350 1 resident
run bulk64 X=1 -- 64 1350 1 resident
run t64_w32 QGCM_RESIDENT_WORKERS=32 -- 64 1350 0 resident
run t256_w64 QGCM_RESIDENT_WORKERS=64 QGCM_RESIDENT_SLOTS=8 -- 256 1350 0 resident
run t64_spin64 QGCM_RESIDENT_SPINNERS=64 -- 64 1350 0 resident
run t16_spin2 QGCM_RESIDENT_SPINNERS=2 -- 16 1350 0 resident
run p64 X=1 -- 1 64 0 resident
run p9000 X=1 -- 1 9000 0 resident
run launch16 X=1 -- 16 1350 1 launch
echo done >> $OUT/sweep.txt
