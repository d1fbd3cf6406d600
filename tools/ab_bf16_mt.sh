#!/bin/bash
# bf16 direct-conv tile A/B (GPU box): BM 128 vs 256 on the layer1/layer2 shapes of 30 clips.
set -e
cd "$(dirname "$0")/.."
bash tools/convbench.sh build
B=gpurun_out/convbench
for mt in 2 4; do
  export CB_BF16=1 CB_MT=$mt
  echo "MT=$mt"
  timeout -k 5 60 $B sp 30 32 56 56 64 160 20
  timeout -k 5 60 $B tp 30 32 56 56 160 64 20
  timeout -k 5 60 $B sp 30 16 28 28 128 288 20
  timeout -k 5 60 $B tp 30 16 28 28 288 128 20
  timeout -k 5 60 $B sp 30 8 14 14 256 576 20
  timeout -k 5 60 $B tp 30 8 14 14 576 256 20
  CB_STRIDE=1 timeout -k 5 60 $B sp 30 32 56 56 64 288 20
done
