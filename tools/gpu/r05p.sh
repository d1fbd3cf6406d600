#!/bin/bash
# round 5: decoder tile rows A/B in the forward (bench with and without CLASFV_DECODER_ROWS8, twice,
# alternated) and the decoder / wide-block tests
out=${1:-gpurun_out/r05p}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "decoder or wino4w" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export CLASFV_DECODER_ROWS8=1; else unset CLASFV_DECODER_ROWS8; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --parity-random 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --extra-c2-ragged 0 > $out/bench_${rep}_$v.json 2> $out/bench_${rep}_$v.err || { echo "bench failed"; tail -20 $out/bench_${rep}_$v.err; exit 1; }
    python -c "
import json; d=json.loads(open('$out/bench_${rep}_$v.json').read().strip().splitlines()[-1]); k=d['kernels']['kernels']
print('rows8=$v', d['value'], d['ms_per_step'], 'decoder ms/fwd', round(k['decoder_kernel']['ms']/k['decoder_kernel']['launches'],4))
"
  done
done
