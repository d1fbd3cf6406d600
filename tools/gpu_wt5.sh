#!/bin/bash
# conv_winot5 before / after (tools/bin/convbench_old = previous build) on layer1 / layer2 temporal
# shapes, channels-last input; CB_CHECK: ko 500 (conv_winot5) vs ko 0 (conv_winot reference) bitwise
out=${1:-gpurun_out/wt5}; mkdir -p $out; export TMPDIR=/tmp CB_NORES=1 CB_CHECK=1
for b in convbench_old convbench; do
  echo "== $b" >> $out/wt5.log
  timeout -k 10 120 tools/bin/$b winot 30 32 56 56 144 64 20 0 500 >> $out/wt5.log 2>&1 || { cat $out/wt5.log; exit 1; }
  timeout -k 10 120 tools/bin/$b winot 30 16 28 28 288 128 20 0 500 >> $out/wt5.log 2>&1 || { cat $out/wt5.log; exit 1; }
done
cat $out/wt5.log
