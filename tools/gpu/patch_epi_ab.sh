#!/bin/bash
# same-box A/B of conv_patch_bf16's epilogue loads: A = tools/bin/convbench_old (generic-pointer loads,
# serialized), B = tools/bin/convbench (global-address-space loads, batched); A B A per shape
out=${1:-gpurun_out/patch_epi_ab}; mkdir -p $out; export TMPDIR=/tmp
for res in 1 0; do
  if [ $res = 1 ]; then export CB_NORES=1; else unset CB_NORES; fi
  for shp in "tpp 30 16 28 28 288 128" "tpp 30 16 28 28 256 128" "tpp 30 8 14 14 576 256" "tpp 30 4 7 7 1152 512" "spp 30 4 7 7 512 1152"; do
    for b in convbench_old convbench convbench_old convbench; do
      echo -n "$b " >> $out/cb.txt
      timeout -k 10 120 tools/bin/$b $shp 20 0 >> $out/cb.txt 2>&1 || { echo "cb $shp failed"; tail $out/cb.txt; exit 1; }
    done
  done
done
cat $out/cb.txt
