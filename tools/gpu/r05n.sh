#!/bin/bash
# round 5: conv_wino4r knock-outs + 6-stage ring, 16-row decoder tiles, packed conv_winot5 transform
# (A/B against tools/bin/convbench_old), then the engine tests and a bench
out=${1:-gpurun_out/r05n}; mkdir -p $out
bash tools/gpu/w4r_ko.sh $out && bash tools/gpu/dec16.sh $out && bash tools/gpu/winot_ab.sh $out && bash tools/gpu/w4r_int.sh $out
