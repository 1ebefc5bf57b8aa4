#!/bin/bash
# Profiles bench.py on the GPU box: kernel trace + stats, then PMC passes (one counter group per
# run, never combined with other trace domains).  Usage: bash tools/profile.sh <tag> [bench args]
set -u
TAG=${1:-r1}; shift || true
ARGS=${*:-"--no-cpu-baseline --no-extra --steps 100"}  # 100 timed steps after 10 warmup (tools/trace_summary.py default)
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run trace --kernel-trace --stats || exit 1
run pmc_sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run pmc_sq2 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE || exit 1
run pmc_fetch --pmc FETCH_SIZE || exit 1
run pmc_write --pmc WRITE_SIZE || exit 1
echo done
