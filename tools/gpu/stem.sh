#!/bin/bash
# conv_stem_x3 variants (persistent over 256-voxel items):
# forward tests, then a bench line and a kernel trace. usage: bash tools/gpu/stem.sh OUTDIR
out=${1:-gpurun_out/stem}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "stem or forward_full or golden or batch_is_per_clip or config3 or x3" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
B="bench.py --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0"
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --extra-bf16 0 --extra-stream 0 > $out/bench.log 2>&1 || { echo "bench failed"; tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $out/trace -o t -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/summary.txt
head -10 $out/summary.txt; sed -n '/per-dispatch/,/^$/p' $out/summary.txt | sed -n '12,20p'
