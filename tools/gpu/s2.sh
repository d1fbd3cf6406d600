#!/bin/bash
# conv_patch_s2_bf16 (polyphase stride-2 patch) vs conv_dma_w on the bf16 strided 1x3x3 convs
# (convbench, 30 clips; CB_CHECK: max |diff| vs conv_dma_w), the bf16 GPU tests, a bench line
out=${1:-gpurun_out/s2}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_BF16=1 CB_NORES=1 CB_STRIDE=2 CB_CHECK=1
for shp in "30 32 56 56 64 256" "30 16 28 28 128 480" "30 8 14 14 256 960"; do
  timeout -k 10 120 $CB sp $shp 10 7400 8220 8320 8210 8310 >> $out/cb.txt 2>&1 || { echo "cb $shp failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
unset CB_BF16 CB_NORES CB_STRIDE CB_CHECK
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "bf16 or config4" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u bench.py --extra-c3 0 --extra-stream 0 --cpu-baseline 0 > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 - $out/bench.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
b=d['bf16']
print('fp32', d['value'], 'bf16', b['value'], b['ms_per_step'], 'deep fp32', d['parity_deep_weights'], '\nbf16 deep', b['parity_vs_cpu_deep_weights'])
for k,v in sorted(b['kernels']['kernels'].items(), key=lambda kv:-kv[1]['ms']): print(f"bf16 {k:22s} {v['ms']:8.3f} ms/10 steps {v['launches']:4d} launches {v['issued_frac_of_pipe_peak']}")
PY
