#!/bin/bash
# conv_wino4w A/B: knock-outs of the current build (layer1, layer2)
out=${1:-gpurun_out/w4w_ab}; mkdir -p $out
CB=tools/bin/convbench
timeout -k 10 120 $CB wino4w 30 32 56 56 64 144 10 0 4 128 0 > $out/cb.txt 2>&1 || { echo fail; cat $out/cb.txt; exit 1; }
timeout -k 10 120 $CB wino4 30 32 56 56 64 144 10 0 4 >> $out/cb.txt 2>&1 || { echo fail; cat $out/cb.txt; exit 1; }
cat $out/cb.txt
