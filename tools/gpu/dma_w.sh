#!/bin/bash
# bf16 direct convs: conv_dma (64-B rows, ko 7300) vs conv_dma_w (128-B rows; 7400 two stages, 7401
# three), bitwise check of every variant against the first (CB_CHECK)
out=${1:-gpurun_out/dma_w}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_BF16=1 CB_NORES=1 CB_CHECK=1
CB_STRIDE=2 CB_NT=8 timeout -k 10 120 $CB sp 30 32 56 56 64 256 10 7300 7400 7401 >> $out/cb.txt 2>&1 || { echo "cb l2 failed"; tail $out/cb.txt; exit 1; }
CB_STRIDE=2 CB_NT=6 timeout -k 10 120 $CB sp 30 16 28 28 128 480 10 7300 7400 7401 >> $out/cb.txt 2>&1 || { echo "cb l3 failed"; tail $out/cb.txt; exit 1; }
CB_STRIDE=2 CB_NT=8 timeout -k 10 120 $CB tp 30 32 28 28 256 128 10 7300 7400 7401 >> $out/cb.txt 2>&1 || { echo "cb l2 tp failed"; tail $out/cb.txt; exit 1; }
unset CB_NORES
CB_STRIDE=2 CB_NT=8 timeout -k 10 120 $CB sp 30 8 14 14 256 928 10 7300 7400 >> $out/cb.txt 2>&1 || true
cat $out/cb.txt
