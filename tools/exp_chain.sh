#!/bin/bash
# Config 5 (tools/bench_configs.py config5) by chain chunk size and codec thread count.
set -u
OUT=gpurun_out/${1:-exp_chain}
mkdir -p $OUT
for mb in 32 64 128 256; do
  for th in 16 14; do
    echo "== chunk ${mb} MiB threads $th" >> $OUT/chain.txt
    QGCM_CHAIN_CHUNK_MB=$mb timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0, 'tools'); sys.path.insert(0, '.')
import json, bench_configs as B
print(json.dumps(B.config5(reps=3, threads=$th)))" >> $OUT/chain.txt 2>> $OUT/chain.err
    rc=$?; if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
