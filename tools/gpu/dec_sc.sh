#!/bin/bash
# decoder: packed-f32 (v_pk_fma/v_pk_mul) vs single-lane v_fma_f32 / v_mul_f32 interpolation and staging
# blend (ko + 32); CB_X3=1 = the fp32 engines' decoder, CB_BF16=1 the bf16 engines'
# usage (GPU box): bash tools/gpu/dec_sc.sh OUTDIR
out=${1:-gpurun_out/dec_sc}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for r in 1 2; do
CB_X3=1 timeout -k 10 120 $CB dec 30 32 112 112 20 0 32 16 48 >> $out/dec.txt 2>&1 || { echo "dec failed"; tail $out/dec.txt; exit 1; }
CB_BF16=1 timeout -k 10 120 $CB dec 30 32 112 112 20 0 32 >> $out/dec.txt 2>&1 || { echo "dec bf16 failed"; tail $out/dec.txt; exit 1; }
done
cat $out/dec.txt
