#!/bin/bash
# conv_winot5 NT 4 (product, 2 waves per SIMD) vs NT 2 at 2 (ko 502) and 3 (ko 503) waves per SIMD
out=${1:-gpurun_out/winot_nt2}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 144 64" "30 16 28 28 288 128"; do
  CB_C8=1 CB_NORES=1 CB_CHECK=1 timeout -k 10 60 $CB winot $shape 20 500 502 503 >> $out/cb.txt 2>&1 || { echo "$shape failed"; tail $out/cb.txt; exit 1; }
  CB_C8=1 CB_CHECK=1 timeout -k 10 60 $CB winot $shape 20 500 502 503 >> $out/cb.txt 2>&1 || { echo "res $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
