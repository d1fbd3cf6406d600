#!/bin/bash
# config[2] with two steps in flight (and --inflight 1 for the A/B), then the bench-driving GPU tests
out=${1:-gpurun_out/c2_inflight}; mkdir -p $out; export TMPDIR=/tmp
for k in 2 1 2; do
timeout -k 10 400 python -u bench.py --workload c2 --steps 5 --warmup 2 --inflight $k > $out/bench_c2_$k.log 2>&1 || { echo "bench c2 failed"; tail -30 $out/bench_c2_$k.log; exit 1; }
tail -1 $out/bench_c2_$k.log | cut -c1-220
done
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "bench or config2 or ranks" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
