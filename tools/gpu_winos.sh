#!/bin/bash
# conv_wino_s (warp-specialised) vs conv_wino_q: convbench timing + bitwise check, then the engine's
# bit-exactness tests and a short bench. usage (GPU box): bash tools/gpu_winos.sh OUTDIR
out=${1:-gpurun_out/winos}; mkdir -p $out; export TMPDIR=/tmp
B=tools/bin/convbench
export CB_CHECK=1
for args in "30 32 56 56 64 144" "30 32 56 56 64 144 res" "4 64 112 112 128 288"; do
  set -- $args
  if [ "$7" = "res" ]; then unset CB_NORES; else export CB_NORES=1; fi
  timeout -k 5 90 $B winoq $1 $2 $3 $4 $5 $6 10 0 7 >> $out/convbench.txt 2>&1 || { echo "convbench failed: $args"; tail -5 $out/convbench.txt; exit 1; }
done
cat $out/convbench.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "bitexact or northstar_config1 or forward_vs_oracle or forward_full_clip or config3" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 > $out/bench.log 2>&1 || { echo "bench failed"; tail -20 $out/bench.log; exit 1; }
python3 -c "
import json; l=json.loads(open('$out/bench.log').read().strip().split('\n')[-1])
print(l['value'], l['ms_per_step'], json.dumps(l['roofline'])[:300]); print({k: (v['launches'], v['ms']) for k, v in l['kernels'].items()})"
