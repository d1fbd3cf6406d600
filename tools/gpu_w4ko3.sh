#!/bin/bash
# conv_wino4 knock-outs on the layer1 shape (8 and 16 chunks): 1 transform, 2 U reloads, 4 epilogue,
# 8 DMAs, 15 all four, 32 barrier, 47 all
out=${1:-gpurun_out/w4ko3}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
{ timeout -k 10 200 $cb wino4 30 32 56 56 64 144 20 0 1 16 2 4 8 15 &&
  timeout -k 10 200 $cb wino4 30 32 56 56 128 144 20 0 1 16 2 4 8 15; } > $out/ko.txt 2>&1 || { echo "ko failed"; cat $out/ko.txt; exit 1; }
cat $out/ko.txt
