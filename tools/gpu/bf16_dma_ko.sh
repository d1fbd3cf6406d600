#!/bin/bash
# bf16 engines' conv_dma knock-outs (convbench ko 7300 + KO: 1 pointer DMAs, 4 no loop DMAs, 8 no
# waits / barriers, 16 no MFMAs) on layer2 / layer3 SP1 (strided 1x3x3) at the product tiles
out=${1:-gpurun_out/bf16_dma_ko}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_BF16=1 CB_STRIDE=2 CB_NORES=1
CB_NT=8 timeout -k 10 120 $CB sp 30 32 56 56 64 256 10 7300 7301 7304 7308 7316 7312 7328 >> $out/cb.txt 2>&1 || { echo "cb l2 failed"; tail $out/cb.txt; exit 1; }
CB_NT=6 timeout -k 10 120 $CB sp 30 16 28 28 128 480 10 7300 7301 7304 7308 7316 7312 7328 >> $out/cb.txt 2>&1 || { echo "cb l3 failed"; tail $out/cb.txt; exit 1; }
cat $out/cb.txt
