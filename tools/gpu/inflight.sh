#!/bin/bash
# bench c1 with 1, 2, 3 steps in flight on round-robin streams (A B A), fp32 + bf16 lines, no extras
out=${1:-gpurun_out/inflight}; mkdir -p $out; export TMPDIR=/tmp
for k in 1 2 3 1 2; do
  timeout -k 10 300 python -u bench.py --inflight $k --steps 20 --extra-c3 0 --extra-stream 0 --cpu-baseline 0 --parity-random 0 > $out/bench_$k.log 2>&1 || { echo "bench $k failed"; tail -30 $out/bench_$k.log; exit 1; }
  python3 - $out/bench_$k.log $k <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('inflight', sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'dice', d.get('dice_delta_vs_cpu'), 'bf16', d['bf16'] and d['bf16']['value'], d['bf16'] and d['bf16']['dice_delta_vs_fp32_fused_masks'], 'frac', d['roofline']['frac'])
PY
done
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "concurrent_streams or two_streams or per_clip" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
