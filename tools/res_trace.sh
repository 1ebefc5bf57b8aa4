#!/bin/bash
# Device-side timeline of the resident kernel: a QGCM_RES_TRACE side build of libqgcm.so in
# ablib/trace/ (built on the CPU side) loaded by tools/bin/per_packet_bench through
# LD_LIBRARY_PATH (its RUNPATH comes after it): mean device-clock microseconds per request from the poll
# that found it to its input staged in LDS, to its result computed, to the result writes acknowledged.
set -u
OUT=gpurun_out/${1:-res_trace}
mkdir -p $OUT
for args in "1 64 1.5 0 resident" "1 1350 1.5 0 resident" "1 9000 1.5 0 resident" "16 1350 1.5 0 resident"; do
  LD_LIBRARY_PATH=$PWD/ablib/trace timeout -k 10 60 tools/bin/per_packet_bench $args >> $OUT/trace.jsonl 2>> $OUT/trace.err
  rc=$?
  echo "$args rc=$rc" >> $OUT/trace.err
  if [ $rc -ge 124 ]; then exit $rc; fi
done
