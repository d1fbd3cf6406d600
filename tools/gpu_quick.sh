#!/bin/bash
# Quick GPU-box iteration: selected GPU tests (pytest -k EXPR), a short fp32 bench line, a kernel-trace
# summary and the FETCH/WRITE passes of the fp32 forward.
# usage (GPU box): bash tools/gpu_quick.sh OUTDIR "pytest -k expression"
out=${1:-gpurun_out/quick}; kexpr=${2:-c8 or bitexact or northstar}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$kexpr" > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
B="bench.py --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -T -d $out/trace -o t -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed"; tail -30 $out/trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -T -d $out/$c -o p -- python3 $B > $out/$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $out/$c.log; exit 1; }
done
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) $(find $out/FETCH_SIZE -name 'p_results.db' | head -1) $(find $out/WRITE_SIZE -name 'p_results.db' | head -1) > $out/summary.txt
find $out/trace -name 't_kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
head -12 $out/summary.txt; grep -A9 "^FETCH_SIZE" $out/summary.txt
