#!/bin/bash
# non-temporal output stores, forward A/B: conv_dma_x3 (fp32 bench) and conv_patch32_bf16 (bf16 bench)
out=${1:-gpurun_out/ntab3}; mkdir -p $out; export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0"
for rep in 1 2; do
for v in base dma bf16base bf16patch; do
  unset CLASFV_DMA_NT_STORES CLASFV_PATCH_NT_STORES
  A="$B"
  [ $v = dma ] && export CLASFV_DMA_NT_STORES=1
  [ $v = bf16base ] && A="$B --dtype bf16"
  [ $v = bf16patch ] && A="$B --dtype bf16" && export CLASFV_PATCH_NT_STORES=1
  timeout -k 10 300 python -u $A > $out/bench_$v.json 2> $out/bench_$v.err || { echo "bench $v failed"; tail -20 $out/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print('$v', d['value'], d['ms_per_step'], {n: round(x['ms']/20,4) for n, x in k.items() if x['ms'] > 5})
" | tee -a $out/ab.txt
done
done
unset CLASFV_DMA_NT_STORES CLASFV_PATCH_NT_STORES
