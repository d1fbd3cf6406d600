#!/bin/bash
# decoder source-index table + host-split bf16 W2 pieces vs the per-wave forms (ko 64: per-wave index
# arithmetic, ko 128: bf16 W2 split in the kernel); bit-identity checks, A B A B timing; then the
# decoder / forward GPU tests and the default bench line
out=${1:-gpurun_out/dec_idx}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for r in 1 2; do
CB_X3=1 timeout -k 10 120 $CB dec 30 32 112 112 20 0 64 0 64 >> $out/dec.txt 2>&1 || { echo "dec x3 failed"; tail $out/dec.txt; exit 1; }
CB_BF16=1 timeout -k 10 120 $CB dec 30 32 112 112 20 0 192 64 128 0 >> $out/dec.txt 2>&1 || { echo "dec bf16 failed"; tail $out/dec.txt; exit 1; }
done
timeout -k 10 120 $CB dec 30 32 112 112 20 0 64 >> $out/dec.txt 2>&1 || { echo "dec f32 failed"; tail $out/dec.txt; exit 1; }
CB_X3=1 timeout -k 10 120 $CB dec 4 64 224 224 10 0 64 >> $out/dec.txt 2>&1 || { echo "dec c3 failed"; tail $out/dec.txt; exit 1; }
cat $out/dec.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "decoder or forward or golden or bf16 or northstar or smoke" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
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
