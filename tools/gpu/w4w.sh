#!/bin/bash
# conv_wino4w bring-up: bit-exactness vs conv_wino4 through the engine, then per-shape timings (convbench)
# usage (GPU box): bash tools/gpu/w4w.sh OUTDIR
out=${1:-gpurun_out/w4w}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "wino4w or wino4_matches or forward_small or forward_full or batch_is_per_clip" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288" "30 16 28 28 128 240" "30 8 14 14 256 480" "30 8 14 14 256 576"; do
  timeout -k 10 120 $CB wino4 $shape 10 >> $out/cb.txt 2>&1 || { echo "cb wino4 $shape failed"; tail $out/cb.txt; exit 1; }
  timeout -k 10 120 $CB wino4w $shape 10 >> $out/cb.txt 2>&1 || { echo "cb wino4w $shape failed"; tail $out/cb.txt; exit 1; }
done
timeout -k 10 120 $CB wino4w 30 32 56 56 64 144 10 0 1 2 4 8 15 >> $out/cb.txt 2>&1 || { echo "cb ko failed"; tail $out/cb.txt; exit 1; }
cat $out/cb.txt
