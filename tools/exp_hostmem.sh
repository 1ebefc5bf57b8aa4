#!/bin/bash
# tools/microbench/hostmem.hip over the access forms and both allocations (resident-kernel design).
OUT=gpurun_out/${1:-hostmem}
mkdir -p $OUT
for f in ${FORMS:-0 1 2 3 4 5 6 7}; do
  for c in 1 0; do
    for b in 64 1408 9040; do
      timeout -k 5 60 tools/bin/hostmem $f $c $b 5000 >> $OUT/hostmem.jsonl 2>&1
      rc=$?
      if [ $rc -ge 124 ]; then echo "stop rc=$rc at $f $c $b" >> $OUT/hostmem.jsonl; exit $rc; fi
    done
  done
done
