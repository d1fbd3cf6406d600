#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 --pmc pass per counter group).
# usage (GPU box): bash tools/pmc.sh OUTDIR [fp32|bf16]
out=$1; dt=${2:-fp32}; mkdir -p $out; export TMPDIR=/tmp
groups=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
 "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
 "TCC_HIT_sum TCC_MISS_sum"
 "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"
 "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $g -T -d $out/g$i -o p -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --dtype $dt --extra-bf16 0 --fuse 1 > $out/g$i.log 2>&1 || { echo "group $i failed"; exit 1; }
done
