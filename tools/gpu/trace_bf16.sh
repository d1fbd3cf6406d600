#!/bin/bash
# bf16 config[4] forward kernel trace (--stats) on the current kernels
out=${1:-gpurun_out/trace_bf16}; mkdir -p $out; export TMPDIR=/tmp
A="bench.py --dtype bf16 --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0 --extra-c2-ragged 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $out/trace -o t -- python3 $A > $out/trace.log 2>&1 || { echo "trace failed"; tail -30 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/summary.txt
head -14 $out/summary.txt
