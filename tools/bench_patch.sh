#!/bin/bash
# bf16 patch-staged convs (conv_patch.hip) on the config[1] layer shapes (bf16 channel padding):
# ko 0 = conv_patch, 900 = conv_dma (direct LDS-DMA implicit GEMM), 901 = the round-1 2-frame patch
# kernel (1x3x3 only). CB_CHECK=1 compares each variant with ko 0 (901 is bit-identical: same K
# order and MFMA sequence; conv_dma sums in tap-major order). usage (GPU box): bash tools/bench_patch.sh
B=${B:-tools/bin/convbench}
export CB_CHECK=1
for args in "30 32 56 56 64 160" "30 16 28 28 128 288" "30 8 14 14 256 576" "30 4 7 7 512 1152"; do
  timeout -k 5 120 $B spp $args 10 0 901 900 || exit 1
done
for args in "30 32 56 56 160 64" "30 32 56 56 64 64" "30 16 28 28 288 128" "30 8 14 14 576 256" "30 4 7 7 1152 512"; do
  timeout -k 5 120 $B tpp $args 10 0 900 || exit 1
done
