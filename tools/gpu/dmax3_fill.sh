#!/bin/bash
# conv_dma_x3 N-tile choice vs last-wave fill on the under-filled layer3 strided convs (30 clips)
out=${1:-gpurun_out/dmax3_fill}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for cfg in "2 8 2" "2 4 2" "2 2 2"; do
  CB_X3CFG="$cfg" CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 $CB tp 30 16 14 14 480 256 20 710 >> $out/cb.txt 2>&1 || { echo "tp3 $cfg failed"; tail $out/cb.txt; exit 1; }
  echo "  ^ cfg $cfg" >> $out/cb.txt
done
for cfg in "2 6 2" "2 5 2" "2 3 2"; do
  CB_X3CFG="$cfg" CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 $CB sp 30 16 28 28 128 480 20 710 >> $out/cb.txt 2>&1 || { echo "sp3 $cfg failed"; tail $out/cb.txt; exit 1; }
  echo "  ^ cfg $cfg" >> $out/cb.txt
done
cat $out/cb.txt
