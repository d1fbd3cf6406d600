#!/bin/bash
# conv_dma on the config[1] direct-conv shapes (30 clips): strided SP1 / TP1 of layers 2-4 with the
# engine's tile choice (CB_NT=... forces the N tile).
# usage (GPU box): bash tools/bench_dma.sh   (binary: python tools/build_convbench.py)
B=${B:-tools/bin/convbench}
export CB_NORES=1 CB_STRIDE=1
for shape in "sp 30 32 56 56 64 240" "tp 30 32 28 28 240 128" "sp 30 16 28 28 128 480" "tp 30 16 14 14 480 256" \
             "sp 30 8 14 14 256 960" "tp 30 8 7 7 960 512"; do
  timeout -k 5 60 $B $shape 10 || exit 1
done
