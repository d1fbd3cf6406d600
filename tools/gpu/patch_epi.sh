#!/bin/bash
# conv_patch_bf16 epilogue loads through global-address-space pointers (batched instead of serialized):
# layer2-4 temporal convs (with / without the residual) and layer4's spatial conv, 30 clips, ko 0
out=${1:-gpurun_out/patch_epi}; mkdir -p $out; export TMPDIR=/tmp
for res in 1 0; do
  if [ $res = 1 ]; then export CB_NORES=1; else unset CB_NORES; fi
  for shp in "tpp 30 16 28 28 288 128" "tpp 30 16 28 28 256 128" "tpp 30 8 14 14 576 256" "tpp 30 4 7 7 1152 512" "spp 30 4 7 7 512 1152"; do
    timeout -k 10 120 tools/bin/convbench $shp 20 0 >> $out/cb.txt 2>&1 || { echo "cb $shp failed"; tail $out/cb.txt; exit 1; }
  done
done
cat $out/cb.txt
