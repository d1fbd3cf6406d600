#!/bin/bash
# conv_dma_x3 wave layout: 4 x 1 (WN 1, product) vs 2 x 2 (WN 2) on the fp32 strided convs, outputs checked
out=${1:-gpurun_out/x3wn}; mkdir -p $out; export TMPDIR=/tmp CB_STRIDE=1 CB_CHECK=1
run() { shape="$1"; cfg="$2"; for wn in 1 2; do echo "wn $wn cfg $cfg" >> $out/wn.log; CB_X3WN=$wn CB_X3CFG="$cfg" timeout -k 10 60 tools/bin/convbench $shape 20 0 710 >> $out/wn.log 2>&1 || { echo "failed $shape $wn"; tail -3 $out/wn.log; exit 1; }; done; }
run "sp 30 16 28 28 128 480" "2 6 2"
run "sp 30 8 14 14 256 960" "2 6 2"
run "tp 30 32 28 28 240 128" "2 8 2"
run "tp 30 16 14 14 480 256" "2 8 2"
run "sp 30 32 56 56 64 240" "2 5 2"
cat $out/wn.log
