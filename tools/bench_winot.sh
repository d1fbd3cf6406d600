#!/bin/bash
# Temporal Winograd variants on the config[1] / config[3] shapes: ko 0 = conv_winot (6 waves), 500 =
# conv_winot5 (rolling halo, U in LDS). CB_CHECK=1 compares every variant's output with conv_winot's
# bit for bit. usage (GPU box): bash tools/bench_winot.sh   (binary: python tools/build_convbench.py)
B=${B:-tools/bin/convbench}
export CB_CHECK=1
for args in "30 32 56 56 144 64" "30 32 56 56 48 64" "30 16 28 28 288 128" "30 16 28 28 240 128" \
            "30 8 14 14 576 256" "8 64 112 112 144 64"; do
  timeout -k 5 120 $B winot $args 10 0 502 504 || exit 1
  CB_NORES=1 timeout -k 5 120 $B winot $args 10 0 502 504 || exit 1
done
