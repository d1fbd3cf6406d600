#!/bin/bash
# conv_wino_s timing variants (ko 7 product, 8 + VAR: priorities, stamps, knock-outs) vs conv_wino_q (ko 0)
out=gpurun_out/winos_b; mkdir -p $out
export CB_NORES=1 CB_CHECK=1
timeout -k 5 120 tools/bin/convbench winoq 30 32 56 56 64 144 10 0 7 72 76 96 100 36 44 > $out/convbench.txt 2>&1; rc=$?
cat $out/convbench.txt; exit $rc
