#!/bin/bash
# bf16 stride-1 1x3x3 convs: patch-staged kernel (spp) vs direct LDS-DMA (sp), 30 clips (GPU box).
set -e
cd "$(dirname "$0")/.."
B=gpurun_out/convbench
sh="30 32 56 56 64 160"
CB_BF16=1 CB_NORES=1 timeout -k 5 60 $B sp $sh 20
CB_NORES=1 timeout -k 5 60 $B spp $sh 20
CLASFV_PATCH_NT=10 CB_NORES=1 timeout -k 5 60 $B spp $sh 20
sh="30 32 112 112 64 160"
CB_BF16=1 CB_NORES=1 timeout -k 5 60 $B sp $sh 10
CB_NORES=1 timeout -k 5 60 $B spp $sh 10
