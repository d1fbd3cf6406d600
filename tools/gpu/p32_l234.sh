#!/bin/bash
# conv_patch32_bf16 at forced N tiles (ko 950 + NB) vs conv_patch_bf16 (ko 0) on the bf16 layer2-4 spatial
# 1x3x3 convs (30 clips, no residual; CB_CHECK: bf16 outputs vs conv_patch_bf16)
out=${1:-gpurun_out/p32_l234}; mkdir -p $out; export TMPDIR=/tmp
export CB_NORES=1 CB_CHECK=1
for shp in "30 16 28 28 128 256 20 0 952 954" "30 8 14 14 256 480 20 0 953 955" "30 16 28 28 128 288 20 0 953" "30 8 14 14 256 576 20 0 953"; do
  timeout -k 10 120 tools/bin/convbench spp $shp >> $out/cb.txt 2>&1 || { echo "cb $shp failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
