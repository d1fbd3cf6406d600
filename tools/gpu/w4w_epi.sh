#!/bin/bash
# conv_wino4w epilogue probes: ko 4 (no epilogue), 128 (no output stores), 64 (start stagger, CB_STAGGER units)
out=${1:-gpurun_out/w4w_epi}; mkdir -p $out
CB=tools/bin/convbench
L1="30 32 56 56 64 144"
timeout -k 10 120 $CB wino4w $L1 10 0 4 128 > $out/cb.txt 2>&1 || { echo fail; cat $out/cb.txt; exit 1; }
for st in 1 2 3 5; do
  CB_STAGGER=$st timeout -k 10 120 $CB wino4w $L1 10 64 >> $out/cb.txt 2>&1 || { echo fail; cat $out/cb.txt; exit 1; }
done
CB_STAGGER=2 timeout -k 10 120 $CB wino4w 30 16 28 28 128 288 10 0 64 128 >> $out/cb.txt 2>&1 || { echo fail; cat $out/cb.txt; exit 1; }
cat $out/cb.txt
