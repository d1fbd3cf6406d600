#!/bin/bash
# conv_dma_x3 tile / ring sweep (CB_X3CFG = "MT NT S") on the strided fp32 convs of 30 clips.
out=${1:-gpurun_out/x3cfg}; mkdir -p $out; export TMPDIR=/tmp CB_STRIDE=1
run() { shape="$1"; shift; for c in "$@"; do echo "cfg $c" >> $out/sweep.log; CB_X3CFG="$c" timeout -k 10 60 tools/bin/convbench $shape 20 710 >> $out/sweep.log 2>&1 || { echo "failed: $shape $c"; tail -3 $out/sweep.log; exit 1; }; done; }
run "sp 30 32 56 56 64 240" "2 5 2" "2 3 3" "1 3 3" "1 3 2" "4 3 2"
run "sp 30 16 28 28 128 480" "2 6 2" "2 6 3" "1 6 3" "1 6 2" "2 3 3" "4 6 2" "4 3 2"
run "tp 30 32 28 28 240 128" "2 4 2" "2 4 3" "1 3 3" "4 3 2"
run "sp 30 8 14 14 256 960" "2 6 2" "2 6 3" "1 6 3" "4 6 2"
grep -E "^cfg|ms" $out/sweep.log | paste - - | awk '{print $2,$3,$4,$5,$6,$7,$8,$9,$10,$11,$12,$13,$14,$15}'
