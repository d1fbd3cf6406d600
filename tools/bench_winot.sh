#!/bin/bash
# Temporal Winograd variants on the config[1] shapes (30 clips): ko 0 = conv_winot (6 waves),
# 100 = conv_winot2 (12 waves), 300 / 301 = conv_winot3 (rolling halo; 4 / 8 waves). CB_CHECK=1 compares
# every variant's output with conv_winot's bit for bit.
# usage (GPU box): bash tools/bench_winot.sh   (needs gpurun_out/convbench from tools/convbench.sh build)
B=${B:-tools/bin/convbench}
export CB_CHECK=1
for args in "30 32 56 56 144 64" "30 32 56 56 48 64" "30 16 28 28 288 128" "30 16 28 28 240 128" \
            "30 8 14 14 576 256" "8 64 112 112 144 64"; do
  timeout -k 5 120 $B winot $args 10 0 100 300 || exit 1
  CB_NORES=1 timeout -k 5 120 $B winot $args 10 0 100 300 || exit 1
done
