#!/bin/bash
# conv_wino4w 16-tile groups (ko 0) vs the widest-TC groups (ko 1024), bit-identity (CB_CHECK), then the
# engine tests that pin conv_wino4w. usage (GPU box): bash tools/gpu/w4w_fill16.sh OUTDIR
out=${1:-gpurun_out/w4w_fill16}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 32 56 56 128 144" "8 64 112 112 64 144" "30 16 28 28 128 288"; do
  CB_CHECK=1 timeout -k 10 120 $CB wino4w $shape 10 1024 0 1024 0 >> $out/cb.txt 2>&1 || { echo "cb $shape failed"; tail $out/cb.txt; exit 1; }
done
cat $out/cb.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "wino4 or forward_full or golden or batch_is_per_clip or config3" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
