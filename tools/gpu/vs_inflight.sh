#!/bin/bash
# VideoStream with two videos in flight: its GPU tests, then the default bench line (its 'stream' object)
out=${1:-gpurun_out/vs_inflight}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "stream or cli or pipeline" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 - $out/bench.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('value', d['value'], 'bf16', d['bf16']['value'], 'stream', d['stream']['value'], 'c3', d['config3']['value'], 'frac', d['roofline']['frac'])
PY
