#!/bin/bash
# fp32 engines: conv_dma_x3 with 128-B A rows (product) vs 64-B rows (CLASFV_NO_DMA_W): bit-identity
# tests, then the forward A/B
out=${1:-gpurun_out/x3_wr}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "dma_w or buffer_dmas or x3 or proj or golden" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
B="bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0"
for rep in 1 2 3; do
for v in wr nowr; do
  unset CLASFV_NO_DMA_W
  [ $v = nowr ] && export CLASFV_NO_DMA_W=1
  timeout -k 10 300 python -u $B > $out/bench_$v.json 2> $out/bench_$v.err || { echo "bench $v failed"; tail -20 $out/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print('$v', d['value'], d['ms_per_step'], {n: round(x['ms']/20,4) for n, x in k.items() if x['ms'] > 5})
" | tee -a $out/ab.txt
done
done
unset CLASFV_NO_DMA_W
