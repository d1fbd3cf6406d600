#!/bin/bash
# conv_twalk_bf16 (frame-walking temporal conv) vs conv_patch_bf16 on the bf16 64-channel temporal convs
# (convbench, 30 clips; CB_CHECK: max |diff| vs conv_patch_bf16), the bf16 GPU tests, a bench line
out=${1:-gpurun_out/twalk}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_CHECK=1
for res in 1 0; do
  if [ $res = 1 ]; then export CB_NORES=1; else unset CB_NORES; fi
  for shp in "30 32 56 56 160 64" "30 32 56 56 64 64"; do
    timeout -k 10 120 $CB tpp $shp 10 0 990 >> $out/cb.txt 2>&1 || { echo "cb $shp failed"; tail $out/cb.txt; exit 1; }
  done
done
cat $out/cb.txt
unset CB_NORES CB_CHECK
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "bf16 or config4" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -60 $out/pytest.log | cut -c1-400; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u bench.py --extra-c3 0 --extra-stream 0 --cpu-baseline 0 > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 - $out/bench.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
b=d['bf16']
print('fp32', d['value'], 'bf16', b['value'], b['ms_per_step'], '\nbf16 parity', b['parity_vs_cpu'], '\nbf16 deep', b['parity_vs_cpu_deep_weights'])
for k,v in sorted(b['kernels']['kernels'].items(), key=lambda kv:-kv[1]['ms']): print(f"bf16 {k:22s} {v['ms']:8.3f} ms/10 steps {v['launches']:4d} launches {v['issued_frac_of_pipe_peak']}")
PY
