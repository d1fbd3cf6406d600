#!/bin/bash
# bf16 patch-kernel variants on the layer1 shapes (ko = FR*1000 + S*100 + NT; 0 = product)
out=gpurun_out/patch_sweep; mkdir -p $out
B=tools/bin/convbench
: > $out/sweep.txt
for args in "spp 30 32 56 56 64 160 10 0 2210 2205 4205 4305 2305 2405"; do
  timeout -k 5 120 $B $args >> $out/sweep.txt 2>&1 || echo "fail: $args" >> $out/sweep.txt
done
for args in "tpp 30 32 56 56 160 64 10 0 4304 4204 2304" "tpp 30 32 56 56 64 64 10 0 4304 2304"; do
  timeout -k 5 120 $B $args >> $out/sweep.txt 2>&1 || echo "fail: $args" >> $out/sweep.txt
done
cat $out/sweep.txt
