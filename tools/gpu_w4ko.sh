#!/bin/bash
# conv_wino4 knock-outs and PMC passes on the layer1 shape (GPU box).
# usage: bash tools/gpu_w4ko.sh OUTDIR
out=${1:-gpurun_out/w4ko}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
timeout -k 10 200 $cb wino4 30 32 56 56 64 144 20 0 1 2 3 4 8 15 16 > $out/ko.txt 2>&1 || { echo "ko failed"; cat $out/ko.txt; exit 1; }
CB_CHECK=1 timeout -k 10 120 $cb wino4 30 32 56 56 64 144 5 0 16 >> $out/ko.txt 2>&1 || { echo "check failed"; cat $out/ko.txt; exit 1; }
cat $out/ko.txt
bash tools/pmc_cb.sh $out/pmc wino4 30 32 56 56 64 144 3 0 > $out/pmc.txt 2>&1 || { echo "pmc failed"; cat $out/pmc.txt; exit 1; }
cat $out/pmc.txt
