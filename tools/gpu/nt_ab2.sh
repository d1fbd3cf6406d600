#!/bin/bash
# non-temporal output stores: conv_wino4r NT (default) vs cached (CLASFV_W4R_CACHED_STORES) vs + conv_winot5
# NT (CLASFV_WINOT_NT_STORES), alternated; then the forward / variant tests
out=${1:-gpurun_out/ntab2}; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
for v in base dma; do
  unset CLASFV_W4R_CACHED_STORES CLASFV_WINOT_NT_STORES CLASFV_DMA_NT_STORES
  [ $v = dma ] && export CLASFV_DMA_NT_STORES=1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0 > $out/bench_$v.json 2> $out/bench_$v.err || { echo "bench failed"; tail -20 $out/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print('$v', d['value'], d['ms_per_step'], 'wino4r', round(k['conv_wino4r']['ms']/20,4), 'winot', round(k['conv_winot']['ms']/20,4), 'dma_x3', round(k['conv_dma_x3']['ms']/20,4), 'parity', d['parity']['dice_delta_fused_masks'])
" | tee -a $out/ab.txt
done
done
unset CLASFV_W4R_CACHED_STORES CLASFV_WINOT_NT_STORES CLASFV_DMA_NT_STORES
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "x3 or proj or golden" > $out/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $out/pytest.log
