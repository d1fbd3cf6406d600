#!/bin/bash
# conv_dma_w N tile / ring depth on the bf16 strided convs (ko 7400: 2 stages, 7401: 3)
out=${1:-gpurun_out/dma_w_tiles}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_BF16=1 CB_NORES=1 CB_STRIDE=2
for nt in 8 4; do
  CB_NT=$nt timeout -k 10 120 $CB sp 30 32 56 56 64 256 10 7400 7401 >> $out/cb.txt 2>&1 || { echo "cb l2 $nt failed"; tail $out/cb.txt; exit 1; }
  echo "^ NT $nt (layer2 SP1)" >> $out/cb.txt
done
for nt in 6; do
  CB_NT=$nt timeout -k 10 120 $CB sp 30 16 28 28 128 480 10 7400 7401 >> $out/cb.txt 2>&1 || { echo "cb l3 $nt failed"; tail $out/cb.txt; exit 1; }
  echo "^ NT $nt (layer3 SP1)" >> $out/cb.txt
done
cat $out/cb.txt
