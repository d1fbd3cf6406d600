#!/bin/bash
# conv_wino4w one-item vs two-item blocks (ko 4096): per-shape timings and bitwise check (convbench)
# usage (GPU box): bash tools/gpu/w4w_items.sh OUTDIR
out=${1:-gpurun_out/w4wi}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288" "30 8 14 14 256 576"; do
  CB_CHECK=1 timeout -k 10 120 $CB wino4w $shape 10 0 512 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
