#!/bin/bash
# fp32 engines' decoder at 4 (product) vs 5 waves per SIMD (ko 256), A B A B, 30 clips and config[3]
out=${1:-gpurun_out/dec_w5}; mkdir -p $out; export TMPDIR=/tmp
for r in 1 2; do
CB_X3=1 timeout -k 10 120 tools/bin/convbench dec 30 32 112 112 20 0 256 0 256 >> $out/dec.txt 2>&1 || { echo "dec failed"; tail $out/dec.txt; exit 1; }
done
CB_X3=1 timeout -k 10 120 tools/bin/convbench dec 4 64 224 224 10 0 256 0 256 >> $out/dec.txt 2>&1 || { echo "dec c3 failed"; tail $out/dec.txt; exit 1; }
cat $out/dec.txt
