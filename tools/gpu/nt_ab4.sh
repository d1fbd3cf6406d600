#!/bin/bash
# bf16 forward A/B: conv_patch_bf16 non-temporal output stores, conv_patch32_bf16 cached stores
out=${1:-gpurun_out/ntab4}; mkdir -p $out; export TMPDIR=/tmp
B="bench.py --dtype bf16 --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0"
for rep in 1 2 3; do
for v in base patchnt p32cached; do
  unset CLASFV_PATCH_NT_STORES CLASFV_PATCH32_CACHED_STORES
  [ $v = patchnt ] && export CLASFV_PATCH_NT_STORES=1
  [ $v = p32cached ] && export CLASFV_PATCH32_CACHED_STORES=1
  timeout -k 10 300 python -u $B > $out/bench_$v.json 2> $out/bench_$v.err || { echo "bench $v failed"; tail -20 $out/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print('$v', d['value'], d['ms_per_step'], {n: round(x['ms']/20,4) for n, x in k.items() if x['ms'] > 5})
" | tee -a $out/ab.txt
done
done
unset CLASFV_PATCH_NT_STORES CLASFV_PATCH32_CACHED_STORES
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "bf16 or patch" > $out/pytest.log 2>&1; echo pytest=$? | tee -a $out/ab.txt; tail -3 $out/pytest.log
