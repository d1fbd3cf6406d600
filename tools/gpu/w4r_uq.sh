#!/bin/bash
# conv_wino4r with a 5-deep U ring (ko 0), + software-pipelined window-column reads (ko 160), + two
# columns per scheduling group (ko 32), against conv_wino4w (ko 8192); bitwise check vs ko 0
out=${1:-gpurun_out/w4ruq}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288" "30 8 14 14 256 576"; do
  CB_CHECK=1 timeout -k 10 120 $CB wino4r $shape 10 0 160 32 8192 0 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
