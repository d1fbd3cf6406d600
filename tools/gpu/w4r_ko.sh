#!/bin/bash
# conv_wino4r knock-outs (timing only; see the KO bits of conv_wino4r) on layer1 and layer2 shapes
# usage (GPU box): bash tools/gpu/w4r_ko.sh OUTDIR
out=${1:-gpurun_out/w4rko}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288"; do
  timeout -k 10 120 $CB wino4r $shape 10 0 1 2 8 16 31 4 128 8192 64 512 576 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
