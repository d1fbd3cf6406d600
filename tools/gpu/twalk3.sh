#!/bin/bash
# conv_twalk_bf16: staged stores (1091) and knock-outs (1092 no stores, 1093 no loads, 1094 no MFMAs,
# 1095 neither loads nor stores) vs the first form (1011)
out=${1:-gpurun_out/twalk3}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_NORES=1
CB_CHECK=1 timeout -k 10 120 $CB tpp 30 32 56 56 160 64 10 1011 1091 >> $out/cb.txt 2>&1 || { echo "cb check failed"; tail $out/cb.txt; exit 1; }
timeout -k 10 120 $CB tpp 30 32 56 56 160 64 10 1011 1091 1092 1093 1094 1095 >> $out/cb.txt 2>&1 || { echo "cb 160 failed"; tail $out/cb.txt; exit 1; }
timeout -k 10 120 $CB tpp 30 32 56 56 64 64 10 0 1011 1091 1092 1093 1094 1095 >> $out/cb.txt 2>&1 || { echo "cb 64 failed"; tail $out/cb.txt; exit 1; }
cat $out/cb.txt
