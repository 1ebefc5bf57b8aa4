#!/bin/bash
# Resident per-packet kernel knob sweep (tools/bin/per_packet_bench, resident path only).
set -u
OUT=gpurun_out/${1:-exp_res}
mkdir -p $OUT
run() {  # label, env..., then -- threads payload
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  echo "== $label ${envs[*]} $*" >> $OUT/sweep.txt
  env "${envs[@]}" timeout -k 10 60 tools/bin/per_packet_bench "$1" "$2" 1.5 0 resident >> $OUT/sweep.txt 2>&1
  local rc=$?
  if [ $rc -ge 124 ]; then echo "stop rc=$rc" >> $OUT/sweep.txt; exit $rc; fi
}
run base1 QGCM_RESIDENT_WORKERS=16 -- 1 1350
run longlife1 QGCM_RESIDENT_LIFE_US=1000000 QGCM_RESIDENT_IDLE_US=1000000 -- 1 1350
run longlife16 QGCM_RESIDENT_LIFE_US=1000000 QGCM_RESIDENT_IDLE_US=1000000 -- 16 1350
run p64 QGCM_RESIDENT_LIFE_US=1000000 QGCM_RESIDENT_IDLE_US=1000000 -- 1 64
run p9000 QGCM_RESIDENT_LIFE_US=1000000 QGCM_RESIDENT_IDLE_US=1000000 -- 1 9000
run w1 QGCM_RESIDENT_WORKERS=1 QGCM_RESIDENT_LIFE_US=1000000 QGCM_RESIDENT_IDLE_US=1000000 -- 1 1350
run w4 QGCM_RESIDENT_WORKERS=4 QGCM_RESIDENT_LIFE_US=1000000 QGCM_RESIDENT_IDLE_US=1000000 -- 4 1350
run hwq8 GPU_MAX_HW_QUEUES=8 -- 16 1350
echo done >> $OUT/sweep.txt
