#!/bin/bash
# the bench-line parity test (steps in flight), then the full default bench line
out=${1:-gpurun_out/parity_fix}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 450 python -u -m pytest tests/test_gpu.py -x -v --timeout 400 --timeout-method thread -k "bench_c1_line_parity or concurrent_streams" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 - $out/bench.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
b=d['bf16']
print('value', d['value'], 'bf16', b['value'], 'stream', d['stream']['value'], 'c3', d['config3']['value'], 'frac', d['roofline']['frac'])
for n,p in [('fp32',d['parity']),('fp32 rnd',d['parity_random_weights']),('fp32 deep',d['parity_deep_weights']),('bf16',b['parity_vs_cpu']),('bf16 rnd',b['parity_vs_cpu_random_weights']),('bf16 deep',b['parity_vs_cpu_deep_weights'])]:
    print(n, p['dice_delta_fused_masks'], p['within_bar'], p['ed_es_pairs_equal'], p['ef_delta_max_per_systole'])
PY
