#!/bin/bash
# Profiles the config-3 workload (tools/bench_configs.py config3: 2^20 x U{64..9000} B, 1024 keys,
# descriptor batches) on the GPU box: kernel trace + stats, then PMC passes (one counter group per
# run, never combined with other trace domains).  Usage: bash tools/profile_config3.sh <tag>
# Summarise with: python tools/pmc_config3.py gpurun_out/prof_c3_<tag>
set -u
TAG=${1:-r2}
OUT=gpurun_out/prof_c3_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 tools/bench_configs.py config3 > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run trace --kernel-trace --stats || exit 1
run pmc_sq2 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE || exit 1
run pmc_fetch --pmc FETCH_SIZE || exit 1
run pmc_write --pmc WRITE_SIZE || exit 1
echo done
