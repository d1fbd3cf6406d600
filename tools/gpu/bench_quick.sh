#!/bin/bash
# default bench line only (no extras) + the fp32 forward tests that pin the changed kernels
out=${1:-gpurun_out/bq}; mkdir -p $out; export TMPDIR=/tmp
K=${2:-"forward or wino4 or x3 or proj or c8 or per_clip or northstar_config1"}
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "$K" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u bench.py --extra-c3 0 --extra-stream 0 --cpu-baseline 0 > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 - $out/bench.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'bf16', d['bf16'] and d['bf16']['value'])
for k,v in sorted(d['kernels']['kernels'].items(), key=lambda kv:-kv[1]['ms']): print(f"{k:22s} {v['ms']:8.3f} ms/10 steps  {v['launches']:4d} launches")
if d['bf16']:
    for k,v in sorted(d['bf16']['kernels']['kernels'].items(), key=lambda kv:-kv[1]['ms']): print(f"bf16 {k:22s} {v['ms']:8.3f}")
PY
