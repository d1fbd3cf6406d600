#!/bin/bash
# decoder_kernel knock-outs at 30 clips (fp32 engines' split-bf16 comb_2: CB_X3): 0 product, 2 no
# comb_2 / head MFMAs, 3 no interpolation. usage (GPU box): bash tools/gpu/dec_ko.sh OUTDIR
out=${1:-gpurun_out/dec_ko}; mkdir -p $out; export TMPDIR=/tmp
CB_X3=1 timeout -k 10 120 tools/bin/convbench dec 30 32 112 112 20 0 2 3 0 >> $out/cb.txt 2>&1 || { echo "cb failed"; tail $out/cb.txt; exit 1; }
timeout -k 10 120 tools/bin/convbench dec 30 32 112 112 20 0 2 3 0 >> $out/cb.txt 2>&1 || { echo "cb failed"; tail $out/cb.txt; exit 1; }
cat $out/cb.txt
