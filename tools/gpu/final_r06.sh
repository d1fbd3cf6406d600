#!/bin/bash
# Round-6 end pass, part 1: full GPU tests, smoke, default bench line, config[2] bench
out=${1:-gpurun_out/final}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py --workload c2 --steps 5 --warmup 2 > $out/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -30 $out/bench_c2.log; exit 1; }
tail -1 $out/bench_c2.log | cut -c1-300
