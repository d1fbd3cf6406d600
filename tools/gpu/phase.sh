#!/bin/bash
# two steps in flight with a phase offset: the next step waits until the previous one queued layer L
out=${1:-gpurun_out/phase}; mkdir -p $out; export TMPDIR=/tmp
for L in -1 0 1 2 -1 0 1; do
  timeout -k 10 300 python -u bench.py --phase-layer $L --steps 20 --extra-c3 0 --extra-stream 0 --cpu-baseline 0 --parity-random 0 > $out/bench_$L.log 2>&1 || { echo "bench $L failed"; tail -30 $out/bench_$L.log; exit 1; }
  python3 - $out/bench_$L.log $L <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('phase', sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'dice', d.get('dice_delta_vs_cpu'), 'bf16', d['bf16']['value'], d['bf16']['dice_delta_vs_fp32_fused_masks'])
PY
done
