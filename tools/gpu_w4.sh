#!/bin/bash
# conv_wino4 (F(4x4,3x3)) on the GPU box: isolated timing against conv_wino_q on the layer1 / layer2
# spatial shapes (30 clips), then the GPU parity tests that exercise it.
# usage (GPU box): bash tools/gpu_w4.sh OUTDIR ["pytest -k expression"]
out=${1:-gpurun_out/w4}; kexpr=${2:-wino4 or winograd_path or golden or oracle}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
{
  timeout -k 10 120 $cb wino4 30 32 56 56 64 144 20 &&
  CB_NORES=1 timeout -k 10 120 $cb winoq 30 32 56 56 64 144 20 &&
  timeout -k 10 120 $cb wino4 30 16 28 28 128 288 20 &&
  CB_NORES=1 timeout -k 10 120 $cb winoq 30 16 28 28 128 288 20 &&
  timeout -k 10 120 $cb wino4 30 8 14 14 256 576 20 &&
  CB_NORES=1 timeout -k 10 120 $cb wino 30 8 14 14 256 576 20 &&
  timeout -k 10 120 $cb wino4 30 4 7 7 512 1152 20 &&
  CB_NORES=1 timeout -k 10 120 $cb wino 30 4 7 7 512 1152 20
} > $out/convbench.txt 2>&1 || { echo "convbench failed"; cat $out/convbench.txt; exit 1; }
cat $out/convbench.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$kexpr" > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -5 $out/pytest_gpu.log
