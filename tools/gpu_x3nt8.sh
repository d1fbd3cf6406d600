#!/bin/bash
# conv_dma_x3 N tile 128 (default for Cout % 128 == 0) vs 64 on the temporal strided convs
out=${1:-gpurun_out/x3nt8}; mkdir -p $out; export TMPDIR=/tmp CB_STRIDE=1
for shape in "tp 30 32 28 28 240 128" "tp 30 16 14 14 480 256" "tp 30 8 7 7 960 512"; do
  for c in "" "2 4 2"; do
    ko=710; [ "$shape" = "tp 30 8 7 7 960 512" ] && ko=714
    echo "cfg '$c'" >> $out/nt8.log
    CB_X3CFG="$c" timeout -k 10 60 tools/bin/convbench $shape 20 $ko >> $out/nt8.log 2>&1 || { echo "failed $shape $c"; tail -3 $out/nt8.log; exit 1; }
  done
done
cat $out/nt8.log
# stride-1 convs: the Winograd kernels vs conv_dma_x3 (direct implicit GEMM on split-bf16 MFMAs)
unset CB_STRIDE; export CB_NORES=1
cmp() { timeout -k 10 60 tools/bin/convbench "$@" >> $out/s1.log 2>&1 || { echo "failed $*"; tail -3 $out/s1.log; exit 1; }; }
cmp wino4 30 16 28 28 128 288 20 0
cmp sp 30 16 28 28 128 288 20 710
cmp wino4 30 8 14 14 256 576 20 0
cmp sp 30 8 14 14 256 576 20 710
cmp wino4 30 4 7 7 512 1152 20 0
cmp sp 30 4 7 7 512 1152 20 710 714
cmp winot 30 32 56 56 144 64 20 0
cmp tp 30 32 56 56 144 64 20 710
cmp winot 30 16 28 28 288 128 20 0
cmp tp 30 16 28 28 288 128 20 710
cmp winot 30 8 14 14 576 256 20 0
cmp tp 30 8 14 14 576 256 20 710
cmp winot 30 4 7 7 1152 512 20 0 604
cmp tp 30 4 7 7 1152 512 20 710 714
cat $out/s1.log
