#!/bin/bash
out=${1:-gpurun_out/w4ko3}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
{ timeout -k 10 200 $cb wino4 30 32 56 56 64 144 20 0 15 47 32 &&
  timeout -k 10 200 $cb wino4 30 32 56 56 128 144 20 0 15 47 32; } > $out/ko.txt 2>&1 || { echo "ko failed"; cat $out/ko.txt; exit 1; }
cat $out/ko.txt
