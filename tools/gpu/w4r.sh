#!/bin/bash
# conv_wino4r (12 row waves, 3 per SIMD) against conv_wino4w on the same U values: per-shape timings,
# per-block phase stamps (ko 512 / 8704) and the bitwise check of every variant against wino4r ko 0
# usage (GPU box): bash tools/gpu/w4r.sh OUTDIR
out=${1:-gpurun_out/w4r}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288" "30 8 14 14 256 576"; do
  CB_CHECK=1 timeout -k 10 120 $CB wino4r $shape 10 0 8192 512 8704 4 128 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
