#!/bin/bash
out=${1:-gpurun_out/wtko}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
{ CB_NORES=1 timeout -k 10 200 $cb winot 30 32 56 56 144 64 20 500 801 802 804 808 815 &&
  CB_NORES=1 timeout -k 10 200 $cb winot 30 16 28 28 288 128 20 500 801 802 804 808 815; } > $out/ko.txt 2>&1 || { echo "ko failed"; cat $out/ko.txt; exit 1; }
cat $out/ko.txt
