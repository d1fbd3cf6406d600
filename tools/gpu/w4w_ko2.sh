#!/bin/bash
# conv_wino4w timing knock-outs on the 16-tile groups (KO bits: 1 no transform, 2 no U loads, 4 no
# epilogue, 8 no loop DMAs, 128 epilogue without stores, 256 serial epilogue; results wrong except 0).
# usage (GPU box): bash tools/gpu/w4w_ko2.sh OUTDIR
out=${1:-gpurun_out/w4w_ko2}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288"; do
  timeout -k 10 120 $CB wino4w $shape 10 0 1 2 4 8 128 256 15 0 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
