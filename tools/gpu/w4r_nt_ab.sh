#!/bin/bash
# conv_wino4r non-temporal output stores in the forward: bench with and without CLASFV_W4R_NT_STORES,
# alternated twice, per-kernel times (the consumer conv_winot5 reads the stored tensor next)
out=${1:-gpurun_out/w4rntab}; mkdir -p $out; export TMPDIR=/tmp
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export CLASFV_W4R_NT_STORES=1; else unset CLASFV_W4R_NT_STORES; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0 > $out/bench_$v.json 2> $out/bench_$v.err || { echo "bench failed"; tail -20 $out/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print('nt=$v', d['value'], d['ms_per_step'], 'wino4r', round(k['conv_wino4r']['ms']/20,4), 'winot', round(k['conv_winot']['ms']/20,4), 'parity', d['parity']['dice_delta_fused_masks'])
" | tee -a $out/ab.txt
done
