#!/bin/bash
# fp32 forward kernel trace (rocprofv3 --kernel-trace --stats) of a short bench run and its summary.
# usage (GPU box): bash tools/gpu/trace.sh OUTDIR [bench args...]
out=${1:-gpurun_out/trace}; shift; mkdir -p $out; export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -T -d $out/trace -o t -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed"; tail -30 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/summary.txt
cat $out/summary.txt | head -70
