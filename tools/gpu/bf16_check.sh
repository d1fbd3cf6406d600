#!/bin/bash
# bf16 engines (stem and layer kernels): the bf16 tests, then a bf16 bench line and
# kernel trace. usage (GPU box): bash tools/gpu/bf16_check.sh OUTDIR
out=${1:-gpurun_out/bf16_check}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "bf16 or config4" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
B="bench.py --dtype bf16 --steps 10 --warmup 3 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0"
timeout -k 10 300 python -u $B > $out/bench.log 2>&1 || { echo "bench failed"; tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $out/trace -o t -- python3 bench.py --dtype bf16 --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0 > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/summary.txt
head -12 $out/summary.txt
