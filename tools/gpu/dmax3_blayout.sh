#!/bin/bash
# conv_dma_x3 with the pair-major weight image (tools/bin/convbench) vs the row-major one
# (tools/bin/convbench_old), buffer (710) and pointer (7200) DMA forms, alternated
out=${1:-gpurun_out/blayout}; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
  for b in convbench_old convbench; do
    CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 tools/bin/$b sp 30 32 56 56 64 240 20 710 7200 >> $out/cb.txt 2>&1 || { echo "$b sp2 failed"; tail $out/cb.txt; exit 1; }
    CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 tools/bin/$b tp 30 32 28 28 240 128 20 710 >> $out/cb.txt 2>&1 || { echo "$b tp2 failed"; tail $out/cb.txt; exit 1; }
    CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 tools/bin/$b sp 30 16 28 28 128 480 20 710 >> $out/cb.txt 2>&1 || { echo "$b sp3 failed"; tail $out/cb.txt; exit 1; }
    CB_NORES=1 timeout -k 10 60 tools/bin/$b sp 30 4 7 7 512 1152 20 710 >> $out/cb.txt 2>&1 || { echo "$b sp4 failed"; tail $out/cb.txt; exit 1; }
    echo "  ^ $b" >> $out/cb.txt
  done
done
cat $out/cb.txt
