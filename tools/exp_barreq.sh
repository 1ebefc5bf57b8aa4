#!/bin/bash
# tools/microbench/barreq.hip: request in pinned host memory vs in device memory written over the BAR
set -u
OUT=gpurun_out/${1:-barreq}
mkdir -p $OUT
for b in 64 1408 9040; do
  for m in 0 1; do
    timeout -k 10 60 tools/bin/barreq $m $b 20000 >> $OUT/barreq.jsonl 2>> $OUT/barreq.err
    rc=$?
    echo "mode $m bytes $b rc=$rc" >> $OUT/barreq.err
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
