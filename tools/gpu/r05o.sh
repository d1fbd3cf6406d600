#!/bin/bash
# round 5: conv_wino4r at NTN = 5 (layer2's 240-channel spatial conv) vs conv_wino4, the full GPU
# test suite, and the default bench
out=${1:-gpurun_out/r05o}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for k in wino4r wino4 wino4r wino4; do
  timeout -k 10 60 $CB $k 30 16 28 28 128 240 20 >> $out/cb.txt 2>&1 || { echo "cb $k failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['bf16']['value'])
for k,v in d['kernels']['kernels'].items(): print(k, v['launches'], v['ms'])
"
