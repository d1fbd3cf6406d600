#!/bin/bash
# conv_wino4r start stagger (CB_W4R_STAGGER=ticks,groups; 100-MHz ticks): time and epilogue concurrency
# usage (GPU box): bash tools/gpu/w4r_stagger.sh OUTDIR
out=${1:-gpurun_out/w4r_stagger}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288"; do
for st in 0,1 900,4 450,8 1800,2 600,6 1200,3; do
  echo "== stagger $st" >> $out/cb.txt
  CB_W4R_STAGGER=$st timeout -k 10 120 $CB wino4r $shape 10 0 512 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
done
cat $out/cb.txt
