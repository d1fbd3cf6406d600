#!/bin/bash
# bf16 patch kernels, round 4: conv_patch32_bf16 (ko 950 / direct-store 960) and conv_patch_bf16 with
# LDS-staged stores (ko 0) vs direct stores (ko 10000); CB_CHECK compares every variant's output with
# the first one's. Then the bf16 engine tests (TESTS=0 skips them).
# usage (GPU box): bash tools/gpu/p32.sh OUTDIR
out=${1:-gpurun_out/p32}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
CB_CHECK=1 CB_NORES=1 timeout -k 10 120 $CB spp 30 32 56 56 64 160 10 10000 0 950 960 >> $out/cb.txt 2>&1 || { echo "cb spp l1 failed"; tail $out/cb.txt; exit 1; }
for shape in "30 16 28 28 128 288" "30 8 14 14 256 576" "30 4 7 7 512 1152"; do
  CB_CHECK=1 CB_NORES=1 timeout -k 10 120 $CB spp $shape 10 10000 0 >> $out/cb.txt 2>&1 || { echo "cb spp $shape failed"; tail $out/cb.txt; exit 1; }
done
for shape in "30 32 56 56 160 64" "30 16 28 28 288 128" "30 8 14 14 576 256" "30 32 56 56 64 64"; do
  CB_CHECK=1 timeout -k 10 120 $CB tpp $shape 10 10000 0 >> $out/cb.txt 2>&1 || { echo "cb tpp $shape failed"; tail $out/cb.txt; exit 1; }
  CB_CHECK=1 CB_NORES=1 timeout -k 10 120 $CB tpp $shape 10 10000 0 >> $out/cb.txt 2>&1 || { echo "cb tpp $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
[ "${TESTS:-1}" = 0 ] && exit 0
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "bf16 or config4" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
