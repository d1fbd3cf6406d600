#!/bin/bash
# conv_dma vs conv_dma_x3 (split-bf16 MFMA) on the strided / 1x1x1 fp32 convs of 30 clips of
# 32x112x112 (ko 0 = conv_dma, 710 = conv_dma_x3, 714 = conv_dma_x3 split-K 4; CB_CHECK: max |diff|),
# then the forward GPU tests and a short bench line.
# usage (GPU box): bash tools/gpu_x3.sh OUTDIR ["pytest -k expression"]
out=${1:-gpurun_out/x3}; mkdir -p $out; export TMPDIR=/tmp
export CB_CHECK=1 CB_STRIDE=1
cb() { timeout -k 10 120 tools/bin/convbench "$@" >> $out/convbench.log 2>&1 || { echo "convbench $* failed"; tail -5 $out/convbench.log; exit 1; }; }
cb sp 30 32 56 56 64 240 20 0 710
cb tp 30 32 28 28 240 128 20 0 710
cb sp 30 16 28 28 128 480 20 0 710
cb tp 30 16 14 14 480 256 20 0 710
cb sp 30 8 14 14 256 960 20 0 710
cb tp 30 8 7 7 960 512 20 0 714 704
cat $out/convbench.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${2:-northstar or golden or oracle or bitexact or decoder or forward or model}" > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-300
python3 - $out/bench.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k,v in sorted(d.get("kernels",{}).items(), key=lambda kv:-kv[1].get("ms",0)): print(k, v)
PY
