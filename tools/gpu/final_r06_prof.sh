#!/bin/bash
# Round-6 end pass, part 2: kernel traces + FETCH/WRITE PMC passes of the fp32 / bf16 / config[3]
# forwards and the clock pass (pmc_pass.sh), then conv_patch32_bf16 vs conv_patch_bf16 on the bf16
# layer1 spatial conv at small batches (the per-clip NB rule's cost)
out=${1:-gpurun_out/final_prof}; mkdir -p $out; export TMPDIR=/tmp
bash tools/gpu/pmc_pass.sh $out || exit 1
for n in 1 4 30; do
  timeout -k 10 120 tools/bin/convbench spp $n 32 56 56 64 160 20 0 955 >> $out/patch32_small.txt 2>&1 || { echo "cb failed"; tail $out/patch32_small.txt; exit 1; }
done
cat $out/patch32_small.txt
