#!/bin/bash
# Profiles the device snappy codec on config 5's resident slots (tools/exp_snappy_dev.py: compress,
# seal, open, uncompress of 2^20 x 1350 B): kernel trace + stats, then PMC passes (one counter group
# per run, never combined with other trace domains).  Usage: bash tools/profile_snappy.sh <tag>
set -u
TAG=${1:-snappy}
OUT=gpurun_out/prof_snappy_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 tools/exp_snappy_dev.py 2 > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run trace --kernel-trace --stats || exit 1
run pmc_a --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE || exit 1
run pmc_b --pmc SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE || exit 1
echo done
