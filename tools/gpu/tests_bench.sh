#!/bin/bash
# GPU tests (optionally a -k filter) then the default bench line. usage: bash tools/gpu/tests_bench.sh OUTDIR [KFILTER]
out=${1:-gpurun_out/tb}; mkdir -p $out; export TMPDIR=/tmp
K=${2:+-k "$2"}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-600
