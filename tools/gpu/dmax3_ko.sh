#!/bin/bash
# conv_dma_x3 timing knock-outs (KO bits of conv_dma_x3: 1 no split, 2 no B-piece reads, 4 no loop DMAs,
# 8 no waits / barriers, 16 no epilogue) on the forward's largest strided convs
out=${1:-gpurun_out/dmax3ko}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB sp 30 32 56 56 64 240 20 7200 710 7232 7236 7204 7201 >> $out/cb.txt 2>&1 || { echo "sp2 failed"; tail $out/cb.txt; exit 1; }
CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB tp 30 32 28 28 240 128 20 7200 710 7232 7236 7204 7201 >> $out/cb.txt 2>&1 || { echo "tp2 failed"; tail $out/cb.txt; exit 1; }
CB_CHECK=1 CB_NORES=1 timeout -k 10 120 $CB sp 30 4 7 7 512 1152 20 7200 710 7232 7236 7204 7201 >> $out/cb.txt 2>&1 || { echo "sp4 failed"; tail $out/cb.txt; exit 1; }
cat $out/cb.txt
CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB sp 30 16 28 28 128 480 20 710 >> $out/cb.txt 2>&1 || { echo "sp3 failed"; tail $out/cb.txt; exit 1; }
CLASFV_NO_DMA_BUF=1 CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB sp 30 16 28 28 128 480 20 710 >> $out/cb.txt 2>&1 || { echo "sp3 failed"; tail $out/cb.txt; exit 1; }
