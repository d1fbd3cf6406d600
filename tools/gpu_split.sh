#!/bin/bash
# conv_winot5 split-K on the small temporal grids (layer4 / layer3 at 30 x 32x112x112): 500 = unsplit,
# 6<NT><S> = NT 2 or 4 channels groups, S splits; outputs vs unsplit (differences = summation order)
out=gpurun_out/split; mkdir -p $out
export CB_CHECK=1
timeout -k 5 120 tools/bin/convbench winot 30 4 7 7 1152 512 20 500 622 624 626 628 642 644 648 > $out/l4.txt 2>&1 &&
timeout -k 5 120 tools/bin/convbench winot 30 4 7 7 960 512 20 500 624 628 644 > $out/l4b.txt 2>&1 &&
timeout -k 5 120 tools/bin/convbench winot 30 8 14 14 576 256 20 500 622 642 644 > $out/l3.txt 2>&1; rc=$?
cat $out/*.txt; exit $rc
