#!/bin/bash
# conv_wino4w per-block phase stamps (convbench ko 512): prologue / chunk loop / epilogue / per-CU gaps
out=${1:-gpurun_out/w4ws}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288"; do
  timeout -k 10 120 $CB wino4w $shape 10 0 512 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
