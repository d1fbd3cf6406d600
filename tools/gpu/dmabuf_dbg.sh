#!/bin/bash
out=${1:-gpurun_out/dmabuf}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB sp 30 32 56 56 64 240 20 7200 710 7232 >> $out/cb.txt 2>&1 || { echo "a failed"; tail $out/cb.txt; exit 1; }
CLASFV_NO_DMA_BUF=1 CB_CHECK=1 CB_STRIDE=2 CB_NORES=1 timeout -k 10 120 $CB sp 30 32 56 56 64 240 20 7200 710 7232 >> $out/cb.txt 2>&1 || { echo "b failed"; tail $out/cb.txt; exit 1; }
cat $out/cb.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "x3_convs or kernel_variants or proj_x3 or golden" > $out/pytest.log 2>&1; echo "pytest rc=$?"; tail -15 $out/pytest.log
