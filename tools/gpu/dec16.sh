#!/bin/bash
# decoder tiles: 8 x 16 voxels (4 waves; ko 0) vs 16 x 16 (8 waves; ko 16), product modes and the two
# knock-outs (2 no comb_2 / head MFMAs, 3 no interpolation); CB_X3=1 = the fp32 engines' decoder
# usage (GPU box): bash tools/gpu/dec16.sh OUTDIR
out=${1:-gpurun_out/dec16}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
CB_X3=1 timeout -k 10 120 $CB dec 30 32 112 112 20 0 16 2 18 3 19 >> $out/dec.txt 2>&1 || { echo "dec failed"; tail $out/dec.txt; exit 1; }
CB_BF16=1 timeout -k 10 120 $CB dec 30 32 112 112 20 0 16 >> $out/dec.txt 2>&1 || { echo "dec bf16 failed"; tail $out/dec.txt; exit 1; }
cat $out/dec.txt
