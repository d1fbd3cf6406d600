#!/bin/bash
# conv_twalk_bf16 prefetch depth / waves-per-SIMD forms (ko 990 + 10 PD + W) vs conv_patch_bf16 (ko 0)
out=${1:-gpurun_out/twalk2}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for res in 1 0; do
  if [ $res = 1 ]; then export CB_NORES=1; else unset CB_NORES; fi
  timeout -k 10 120 $CB tpp 30 32 56 56 160 64 10 0 1011 1021 1031 1012 >> $out/cb.txt 2>&1 || { echo "cb 160 failed"; tail $out/cb.txt; exit 1; }
  timeout -k 10 120 $CB tpp 30 32 56 56 64 64 10 0 1011 1021 1031 1012 1022 1032 >> $out/cb.txt 2>&1 || { echo "cb 64 failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
