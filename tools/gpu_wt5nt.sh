#!/bin/bash
# conv_winot5 N tile: 64 channels per wave (504) vs 32 (502, 160 VGPRs: 3 blocks per CU), channels-last input
out=${1:-gpurun_out/wt5nt}; mkdir -p $out; export TMPDIR=/tmp CB_NORES=1
timeout -k 10 120 tools/bin/convbench winot 30 32 56 56 144 64 20 504 502 > $out/nt.log 2>&1 || { cat $out/nt.log; exit 1; }
timeout -k 10 120 tools/bin/convbench winot 30 16 28 28 288 128 20 504 502 >> $out/nt.log 2>&1 || { cat $out/nt.log; exit 1; }
timeout -k 10 120 tools/bin/convbench winot 30 8 14 14 576 256 20 504 502 >> $out/nt.log 2>&1 || { cat $out/nt.log; exit 1; }
cat $out/nt.log
