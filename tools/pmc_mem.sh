#!/bin/bash
# memory-side PMC passes per variant: bash tools/pmc_mem.sh <tag> <variants...>
TAG=$1; shift
OUT=gpurun_out/pmcm_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for v in "$@"; do
  i=0
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    QGCM_VARIANT=$v timeout -k 10 200 rocprofv3 --pmc $P -d $OUT/v${v}_m$i -o p --output-format csv -- python3 tools/run_variant.py > $OUT/v${v}_m$i.log 2>&1 || { echo "fail v$v m$i"; tail -3 $OUT/v${v}_m$i.log; }
  done
  echo "variant $v done"
done
