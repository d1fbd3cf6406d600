#!/bin/bash
# Plumbing kernels (clips, pass labels, fusion): the GPU tests that pin them, a bench line and a trace.
# usage (GPU box): bash tools/gpu/plumb.sh OUTDIR
out=${1:-gpurun_out/plumb}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "clips or label or fuse or pipeline or northstar or stream or sharded or cli" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
B="bench.py --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0"
timeout -k 10 300 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $out/trace -o t -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/summary.txt
grep -E "clips|labels|fuse|pack" $out/summary.txt | head -8
