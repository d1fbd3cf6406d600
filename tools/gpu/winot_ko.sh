#!/bin/bash
# conv_winot5 knock-outs (TS = 4, NT = 4) on layer1's temporal convs, 8-channel-blocked input as in the
# engine: 802 no loop DMAs, 816 no U DMAs, 832 no raw DMAs, 801 no transform, 808 no wait / barrier,
# 804 no epilogue; residual form 817 / 833. usage (GPU box): bash tools/gpu/winot_ko.sh OUTDIR
out=${1:-gpurun_out/winot_ko}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 144 64" "30 16 28 28 288 128"; do
  CB_C8=1 CB_NORES=1 timeout -k 10 60 $CB winot $shape 10 500 802 816 832 801 808 804 500 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
  CB_C8=1 timeout -k 10 60 $CB winot $shape 10 500 817 833 500 >> $out/cb.txt 2>&1 || { echo "cb res $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
