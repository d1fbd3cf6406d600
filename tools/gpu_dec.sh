#!/bin/bash
# Decoder A/B on the GPU box: convbench timings of the fp32 (MFMA f32), X3 (split-bf16, the fp32
# engines' default) and bf16-engine forms, then the decoder / forward GPU tests.
# usage (GPU box): bash tools/gpu_dec.sh OUTDIR
out=${1:-gpurun_out/dec}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 120 tools/bin/convbench dec 30 32 112 112 30 0 2 3 > $out/dec_f32.log 2>&1 || { cat $out/dec_f32.log; exit 1; }
CB_X3=1 timeout -k 10 120 tools/bin/convbench dec 30 32 112 112 30 0 > $out/dec_x3.log 2>&1 || { cat $out/dec_x3.log; exit 1; }
CB_BF16=1 timeout -k 10 120 tools/bin/convbench dec 30 32 112 112 30 0 > $out/dec_bf16.log 2>&1 || { cat $out/dec_bf16.log; exit 1; }
cat $out/dec_f32.log $out/dec_x3.log $out/dec_bf16.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${2:-decoder or northstar or golden}" > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
