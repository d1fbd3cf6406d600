#!/bin/bash
# run_model with two clip batches in flight: the tests that drive multi-batch fusion, then config[2]
out=${1:-gpurun_out/rm_inflight}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "in_flight or concurrent or config2 or config_2 or ranks or stream or fusion or northstar" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for r in 1 2; do
timeout -k 10 400 python -u bench.py --workload c2 --steps 5 --warmup 2 > $out/bench_c2_$r.log 2>&1 || { echo "bench c2 failed"; tail -30 $out/bench_c2_$r.log; exit 1; }
tail -1 $out/bench_c2_$r.log | cut -c1-200
done
