#!/bin/bash
# conv_wino4r in the engine: the wide-block bit-identity tests and the forward / golden tests, then
# the knock-outs (tools/gpu/w4r_ko.sh) and a short bench
# usage (GPU box): bash tools/gpu/w4r_int.sh OUTDIR
out=${1:-gpurun_out/w4ri}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "wino4w or wino4_matches or forward_small or forward_full or golden or batch_is_per_clip or kernel_variants or decoder" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
true
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])
for k,v in d['kernels'].items(): print(k, v['launches'], v['ms'])
"
