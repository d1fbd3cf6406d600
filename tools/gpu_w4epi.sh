#!/bin/bash
# conv_wino4 epilogue probes (layer1 and layer2 shapes, 30 clips): 4 no epilogue, 8192 no output stores,
# 16384 no unit LDS reads, 24576 neither, 32768 the (channel, column, 4 tiles) unit form (correct;
# CB_CHECK: bit-identical expected)
out=${1:-gpurun_out/w4epi}; mkdir -p $out; export TMPDIR=/tmp CB_CHECK=1
timeout -k 10 120 tools/bin/convbench wino4 30 32 56 56 64 144 20 0 4 8192 16384 24576 32768 > $out/epi.log 2>&1 || { cat $out/epi.log; exit 1; }
timeout -k 10 120 tools/bin/convbench wino4 30 16 28 28 128 288 20 0 4 8192 16384 32768 >> $out/epi.log 2>&1 || { cat $out/epi.log; exit 1; }
cat $out/epi.log
