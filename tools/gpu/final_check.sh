#!/bin/bash
# the final library: the full GPU test suite and smoke (no bench)
out=${1:-gpurun_out/final_check}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
