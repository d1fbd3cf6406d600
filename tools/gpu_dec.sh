#!/bin/bash
# decoder variants (30 clips, 32x112x112): product vs the per-row fp32 form, outputs cross-checked
out=gpurun_out/dec; mkdir -p $out
timeout -k 5 120 tools/bin/convbench dec 30 32 112 112 10 0 4 2 3 > $out/dec_f32.txt 2>&1 &&
CB_BF16=1 timeout -k 5 120 tools/bin/convbench dec 30 32 112 112 10 0 > $out/dec_bf16.txt 2>&1; rc=$?
cat $out/dec_f32.txt $out/dec_bf16.txt; exit $rc
