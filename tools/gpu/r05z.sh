#!/bin/bash
out=${1:-gpurun_out/r05z}; mkdir -p $out
bash tools/gpu/dmax3_blayout.sh $out && bash tools/gpu/dmax3_fill.sh $out && bash tools/gpu/winot_fill.sh $out
