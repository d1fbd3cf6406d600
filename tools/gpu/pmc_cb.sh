#!/bin/bash
# PMC passes over one convbench variant (GPU box): SQ timing counters, LDS/instruction mix, HBM bytes.
# usage: bash tools/gpu/pmc_cb.sh OUTDIR convbench-args...   e.g. bash tools/gpu/pmc_cb.sh gpurun_out/p winot 30 32 56 56 144 64 3 300
out=$1; shift; mkdir -p $out; export TMPDIR=/tmp
B=${B:-tools/bin/convbench}
passes=(
 "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
i=0
for c in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d $out/p$i -o p --output-format csv -- $B "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_cb_summary.py $out
