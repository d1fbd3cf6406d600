#!/bin/bash
# conv_wino4w: software-pipelined epilogue (ko 0) vs the serial order (ko 256); bit-identity through
# the engine. usage (GPU box): bash tools/gpu/w4w_epi2.sh OUTDIR
out=${1:-gpurun_out/w4w_epi2}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288" "30 8 14 14 256 576"; do
  CB_CHECK=1 timeout -k 10 120 $CB wino4w $shape 10 256 0 256 0 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "wino4w or forward_full or golden" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
