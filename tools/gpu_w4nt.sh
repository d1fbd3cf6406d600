#!/bin/bash
# conv_wino4 output stores: regular vs non-temporal (ko 65536, bit-identical), layer1 and layer2 shapes
out=${1:-gpurun_out/w4nt}; mkdir -p $out; export TMPDIR=/tmp CB_CHECK=1
timeout -k 10 120 tools/bin/convbench wino4 30 32 56 56 64 144 20 0 65536 > $out/nt.log 2>&1 || { cat $out/nt.log; exit 1; }
timeout -k 10 120 tools/bin/convbench wino4 30 16 28 28 128 288 20 0 65536 >> $out/nt.log 2>&1 || { cat $out/nt.log; exit 1; }
cat $out/nt.log
