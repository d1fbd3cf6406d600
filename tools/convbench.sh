#!/bin/bash
# Build tools/convbench (engine kernels + knock-out variants) and time the layer1 shapes.
# usage (GPU box or build container for the compile only): bash tools/convbench.sh [build]
set -e
cd "$(dirname "$0")/.."
C=fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking_amd/csrc
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCLASFV_KNOCKOUTS -Iinclude -o ${CB_OUT:-gpurun_out/convbench} \
  tools/convbench.hip $C/winograd.hip $C/winograd2.hip $C/winograd3.hip $C/winograd_t.hip $C/conv.hip $C/conv_patch.hip $C/decoder.hip
[ "$1" = build ] && exit 0
B=gpurun_out/convbench
if [ -n "$CB_ARGS" ]; then
  while read -r line; do [ -n "$line" ] && timeout -k 5 120 $B $line; done <<< "$CB_ARGS"
  exit 0
fi
CB_NORES=1 timeout -k 5 120 $B wino 30 32 56 56 64 144 20 0 8 6
CB_NORES=1 timeout -k 5 120 $B winot 30 32 56 56 144 64 20 0 8 6
timeout -k 5 120 $B winot 30 32 56 56 144 64 20 0 8
