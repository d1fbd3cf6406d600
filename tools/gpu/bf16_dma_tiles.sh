#!/bin/bash
# bf16 engines' conv_dma (buffer DMAs) on the strided spatial convs: BM 128 (MT 2) vs 256 (MT 4), N tiles
# usage (GPU box): bash tools/gpu/bf16_dma_tiles.sh OUTDIR
out=${1:-gpurun_out/bf16_dma_tiles}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_BF16=1 CB_STRIDE=2 CB_NORES=1
for cfg in "2 8" "4 8" "2 4" "4 4"; do
  set -- $cfg
  CB_MT=$1 CB_NT=$2 timeout -k 10 120 $CB sp 30 32 56 56 64 256 10 0 >> $out/cb.txt 2>&1 || { echo "cb l2 $cfg failed"; tail $out/cb.txt; exit 1; }
  echo "^ MT $1 NT $2 (layer2 SP1)" >> $out/cb.txt
done
for cfg in "2 6" "4 6" "2 5" "4 5" "2 3" "4 3"; do
  set -- $cfg
  CB_MT=$1 CB_NT=$2 timeout -k 10 120 $CB sp 30 16 28 28 128 480 10 0 >> $out/cb.txt 2>&1 || { echo "cb l3 $cfg failed"; tail $out/cb.txt; exit 1; }
  echo "^ MT $1 NT $2 (layer3 SP1)" >> $out/cb.txt
done
cat $out/cb.txt
