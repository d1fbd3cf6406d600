#!/bin/bash
# conv_dma split-K on layer4's temporal stride-2 conv (30 x 32x112x112: 921 -> 512, T 8 -> 4, 7x7)
out=gpurun_out/split2; mkdir -p $out
export CB_CHECK=1 CB_STRIDE=2 CB_NORES=1
timeout -k 5 120 tools/bin/convbench tp 30 8 7 7 928 512 20 0 702 703 704 706 708 > $out/l4tp.txt 2>&1; rc=$?
cat $out/*.txt; exit $rc
