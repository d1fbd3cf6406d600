#!/bin/bash
out=${1:-gpurun_out/w4rnt}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288" "30 8 14 14 256 576"; do
  CB_CHECK=1 timeout -k 10 120 $CB wino4r $shape 10 0 2048 0 2048 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
