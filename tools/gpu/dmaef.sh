#!/bin/bash
# conv_dma_x3 with compile-time epilogue flags (tools/bin/convbench) vs runtime flags (convbench_old)
out=${1:-gpurun_out/dmaef}; mkdir -p $out
for b in convbench_old convbench; do
  echo "== $b" >> $out/cb.txt
  CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 tools/bin/$b sp 30 32 56 56 64 240 10 710 >> $out/cb.txt 2>&1 || exit 1
  CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 tools/bin/$b tp 30 32 28 28 240 128 10 710 >> $out/cb.txt 2>&1 || exit 1
  CB_STRIDE=2 CB_NORES=1 timeout -k 10 60 tools/bin/$b sp 30 16 28 28 128 480 10 710 >> $out/cb.txt 2>&1 || exit 1
  CB_NORES=1 timeout -k 10 60 tools/bin/$b sp 30 4 7 7 512 1152 10 710 >> $out/cb.txt 2>&1 || exit 1
  CB_NORES=1 timeout -k 10 60 tools/bin/$b pw 30 8 14 14 256 64 10 710 >> $out/cb.txt 2>&1 || exit 1
done
cat $out/cb.txt
