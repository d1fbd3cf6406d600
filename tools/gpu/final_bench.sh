#!/bin/bash
# the default bench line and the config[2] line on the final tree
out=${1:-gpurun_out/final_bench}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py --workload c2 --steps 5 --warmup 2 > $out/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -30 $out/bench_c2.log; exit 1; }
tail -1 $out/bench_c2.log | cut -c1-300
