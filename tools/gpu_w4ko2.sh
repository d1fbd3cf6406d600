#!/bin/bash
# conv_wino4 knock-outs: per-block overhead probe (8 vs 16 chunks per block) on the layer1 map
out=${1:-gpurun_out/w4ko2}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
{ timeout -k 10 200 $cb wino4 30 32 56 56 64 144 20 0 15 4 &&
  timeout -k 10 200 $cb wino4 30 32 56 56 128 144 20 0 15 4 &&
  timeout -k 10 200 $cb wino4 15 32 56 56 128 144 20 0 15 4 &&
  timeout -k 10 200 $cb wino4 30 16 28 28 128 288 20 0 15 4; } > $out/ko.txt 2>&1 || { echo "ko failed"; cat $out/ko.txt; exit 1; }
cat $out/ko.txt
