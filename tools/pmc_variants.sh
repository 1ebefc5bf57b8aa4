#!/bin/bash
# PMC passes for kernel variants: bash tools/pmc_variants.sh <tag> <variants...>
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE"
P2="SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQC_ICACHE_BUSY_CYCLES SQ_WAVES"
P4="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL"
for v in "$@"; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    QGCM_VARIANT=$v timeout -k 10 200 rocprofv3 --pmc $P -d $OUT/v${v}_p$i -o p --output-format csv -- python3 tools/run_variant.py > $OUT/v${v}_p$i.log 2>&1 || { echo "fail v$v p$i"; exit 1; }
  done
  echo "variant $v done"
done
