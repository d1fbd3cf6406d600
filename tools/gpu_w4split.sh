#!/bin/bash
out=${1:-gpurun_out/w4split}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
{ timeout -k 10 200 $cb wino4 30 4 7 7 512 1152 20 0 1002 1004 1008 &&
  timeout -k 10 200 $cb wino4 30 8 14 14 256 576 20 0 1002 1004 &&
  timeout -k 10 200 $cb wino4 30 16 28 28 128 288 20 0 1002 &&
  CB_CHECK=1 timeout -k 10 200 $cb wino4 30 4 7 7 512 1152 3 1001 1002 1004; } > $out/split.txt 2>&1 || { echo "split failed"; cat $out/split.txt; exit 1; }
cat $out/split.txt
