#!/bin/bash
# conv_twalk_bf16 on layer2's 128-output-channel temporal convs (two 64-channel halves per column on one
# XCD) vs conv_patch_bf16 (ko 0): ko 990 = the product launcher, 1000 + 1000 PD + TS = forced forms
out=${1:-gpurun_out/twalk_l2}; mkdir -p $out; export TMPDIR=/tmp
export CB_CHECK=1
for res in 1 0; do
  if [ $res = 1 ]; then export CB_NORES=1; else unset CB_NORES; fi
  for shp in "30 16 28 28 288 128" "30 16 28 28 256 128"; do
    timeout -k 10 120 tools/bin/convbench tpp $shp 20 0 990 2016 3016 2008 3008 >> $out/cb.txt 2>&1 || { echo "cb $shp failed"; tail $out/cb.txt; exit 1; }
  done
done
cat $out/cb.txt
