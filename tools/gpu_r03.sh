#!/bin/bash
# Round-3 GPU pass: full GPU tests, smoke, default bench line, config[2] bench (1 rank), kernel trace.
# usage (GPU box): bash tools/gpu_r03.sh OUTDIR
out=${1:-gpurun_out/r03}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-600
timeout -k 10 400 python -u bench.py --workload c2 --steps 5 --warmup 2 > $out/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -30 $out/bench_c2.log; exit 1; }
tail -1 $out/bench_c2.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -T -d $out/trace -o t -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 > $out/trace.log 2>&1 || { echo "trace failed"; tail -30 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/kernel_summary.txt
head -20 $out/kernel_summary.txt
