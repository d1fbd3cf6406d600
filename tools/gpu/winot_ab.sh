#!/bin/bash
# conv_winot5 A/B: the current build (tools/bin/convbench) vs an older one (tools/bin/convbench_old),
# layer1 / layer2 temporal convs on 8-channel-blocked input, without and with the residual, alternated
out=${1:-gpurun_out/winot_ab}; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
for shape in "30 32 56 56 144 64" "30 16 28 28 288 128"; do
  for b in convbench_old convbench; do
    CB_C8=1 CB_NORES=1 timeout -k 10 60 tools/bin/$b winot $shape 20 500 >> $out/cb.txt 2>&1 || { echo "$b $shape failed"; tail $out/cb.txt; exit 1; }
    echo "  ^ $b" >> $out/cb.txt
    CB_C8=1 timeout -k 10 60 tools/bin/$b winot $shape 20 500 >> $out/cb.txt 2>&1 || { echo "$b res $shape failed"; tail $out/cb.txt; exit 1; }
    echo "  ^ $b" >> $out/cb.txt
  done
done
done
cat $out/cb.txt
