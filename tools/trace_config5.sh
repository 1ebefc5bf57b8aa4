#!/bin/bash
# Kernel + memory-copy trace of config 5 (tools/bench_configs.py config5), no counters: where the
# chained snappy + GCM host pipeline spends its time.  Summarise with tools/chain_timeline.py.
set -u
OUT=gpurun_out/${1:-c5trace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o c5 -- python3 tools/bench_configs.py config5 > $OUT/config5.log 2>&1
echo "trace rc=$?" >> $OUT/steps.txt
