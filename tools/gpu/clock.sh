#!/bin/bash
# Effective clock (GRBM_GUI_ACTIVE / 8 / wall time) and MFMA-pipe occupancy per kernel of the fp32
# bench forward: a kernel-trace pass and a PMC pass (separate runs). usage: bash tools/gpu/clock.sh OUTDIR
out=${1:-gpurun_out/clock}; mkdir -p $out; export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --inflight 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0"
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $out/trace -o t -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -T -d $out/pmc -o p -- python3 $B > $out/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $out/pmc.log; exit 1; }
python3 tools/clock_summary.py $(find $out/trace -name 't_results.db' | head -1) $(find $out/pmc -name 'p_results.db' | head -1) > $out/clock.txt
cat $out/clock.txt
