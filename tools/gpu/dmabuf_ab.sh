#!/bin/bash
# conv_dma_x3 pointer-form (ko 7200) vs buffer-offset (ko 7232) DMAs, and the BUF form's knock-outs
# (7236 no loop DMAs, 7233 no split), then two benches (default, CLASFV_NO_DMA_BUF=1)
out=${1:-gpurun_out/dmabuf}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for rep in 1 2; do
CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB sp 30 32 56 56 64 240 20 7200 7232 7236 7233 >> $out/cb.txt 2>&1 || { echo "sp2 failed"; tail $out/cb.txt; exit 1; }
CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB tp 30 32 28 28 240 128 20 7200 7232 >> $out/cb.txt 2>&1 || { echo "tp2 failed"; tail $out/cb.txt; exit 1; }
CB_CHECK=1 CB_NORES=1 timeout -k 10 120 $CB sp 30 4 7 7 512 1152 20 7200 7232 >> $out/cb.txt 2>&1 || { echo "sp4 failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export CLASFV_NO_DMA_BUF=1; else unset CLASFV_NO_DMA_BUF; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0 > $out/bench_$v.json 2> $out/bench_$v.err || { echo "bench failed"; tail -20 $out/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print('no_dma_buf=$v', d['value'], d['ms_per_step'], 'dma_x3 ms/fwd', round(k['conv_dma_x3']['ms']/10*k['conv_dma_x3']['launches']/k['conv_dma_x3']['launches'],4), 'proj', round(k['conv_proj_x3']['ms'],3))
" | tee -a $out/bench_ab.txt
done
