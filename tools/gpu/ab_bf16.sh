#!/bin/bash
# bf16 config[4] (DTYPE=fp32: the fp32 headline) bench A/B: ENV_A vs ENV_B (environment assignments, e.g. "CLASFV_NO_TWALK=1"), interleaved
# A B A B, each a fresh process; prints value, ms/step and the per-kernel summed ms
out=${1:-gpurun_out/ab_bf16}; A=${2:-}; B=${3:-}; mkdir -p $out; export TMPDIR=/tmp
BA="bench.py --dtype ${DTYPE:-bf16} --extra-bf16 0 --extra-c3 0 --extra-stream 0 --cpu-baseline 0 --parity-random 0 --steps 20 --warmup 3"
i=0
for v in A B A B; do
  i=$((i+1)); E=$A; [ $v = B ] && E=$B
  env $E timeout -k 10 300 python -u $BA > $out/bench_${i}_$v.log 2>&1 || { echo "bench $v failed"; tail -30 $out/bench_${i}_$v.log; exit 1; }
  python3 - $out/bench_${i}_$v.log "$v: $E" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
k=d['kernels']['kernels']
print(sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], ' '.join(f"{n}={v['ms']/d['steps']:.3f}" for n,v in sorted(k.items(), key=lambda kv:-kv[1]['ms'])[:7]), flush=True)
PY
done
