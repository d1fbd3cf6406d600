#!/bin/bash
# One GPU-box pass: gpu tests, default bench line, kernel-trace profile of the bench.
# usage (GPU box): bash tools/gpu_check.sh OUTDIR
out=${1:-gpurun_out/check}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -T -d $out/trace -o t -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 > $out/trace.log 2>&1 || { echo "trace failed"; tail -30 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/kernel_summary.txt
find $out/trace -name '*stats.csv' -exec cp {} $out/ \;
head -20 $out/kernel_summary.txt
