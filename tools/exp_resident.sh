#!/bin/bash
# Resident per-packet kernel experiments (tools/bin/per_packet_bench): thread counts, next to a bulk
# host batch, hardware-queue count and lifetime knobs.
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
run t1 X=1 -- 1 1350 0 resident
run t16 X=1 -- 16 1350 0 resident
run t64 X=1 -- 64 1350 0 resident
run t256 X=1 -- 256 1350 0 resident
run p64 X=1 -- 1 64 0 resident
run p9000 X=1 -- 1 9000 0 resident
run bulk16 X=1 -- 16 1350 1 both
run bulk16_hwq8 GPU_MAX_HW_QUEUES=8 -- 16 1350 1 resident
run bulk16_life500 QGCM_RESIDENT_LIFE_US=500 -- 16 1350 1 resident
echo done >> $OUT/sweep.txt
