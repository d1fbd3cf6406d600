#!/bin/bash
# conv_winot5 channel-block choice by last-wave fill: auto (ko 500) vs NT 4 (504) vs NT 2 at three
# waves per SIMD (503), layer3 / layer2 / layer1 temporal shapes (30 clips)
out=${1:-gpurun_out/winot_fill}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 8 14 14 576 256" "30 16 28 28 288 128" "30 32 56 56 144 64"; do
  CB_C8=1 CB_NORES=1 CB_CHECK=1 timeout -k 10 60 $CB winot $shape 20 504 500 503 >> $out/cb.txt 2>&1 || { echo "$shape failed"; tail $out/cb.txt; exit 1; }
  CB_C8=1 CB_CHECK=1 timeout -k 10 60 $CB winot $shape 20 504 500 503 >> $out/cb.txt 2>&1 || { echo "res $shape failed"; tail $out/cb.txt; exit 1; }
done
CB_NORES=1 CB_CHECK=1 timeout -k 10 60 $CB winot 30 8 14 14 480 256 20 504 500 503 >> $out/cb.txt 2>&1 || { echo "480 failed"; tail $out/cb.txt; exit 1; }
cat $out/cb.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "kernel_variants or golden or forward_full or batch_is_per_clip or x3 or proj" > $out/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $out/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print(d['value'], d['ms_per_step'], 'winot ms/fwd', round(k['conv_winot']['ms']/20,4))
"
