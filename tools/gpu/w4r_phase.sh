#!/bin/bash
# conv_wino4r per-block phase stamps with the cross-CU epilogue concurrency (lockstep check), layer1-3
# usage (GPU box): bash tools/gpu/w4r_phase.sh OUTDIR
out=${1:-gpurun_out/w4r_phase}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288"; do
  timeout -k 10 120 $CB wino4r $shape 10 0 512 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
