#!/bin/bash
# conv_winot5 raw ring 3 / U ring 2 (tools/bin/convbench) vs the 2-stage ring (tools/bin/convbench_old,
# built from the previous tree); 8-channel-blocked input as in the engine; then the engine tests that
# pin the temporal kernels. usage (GPU box): bash tools/gpu/wt3.sh OUTDIR
out=${1:-gpurun_out/wt3}; mkdir -p $out; export TMPDIR=/tmp
for shape in "30 32 56 56 144 64" "30 16 28 28 288 128" "30 8 14 14 576 256" "30 32 56 56 48 64"; do
  for b in convbench_old convbench; do
    echo "$b" >> $out/cb.txt
    CB_C8=1 timeout -k 10 60 tools/bin/$b winot $shape 10 500 >> $out/cb.txt 2>&1 || { echo "cb $b $shape failed"; tail $out/cb.txt; exit 1; }
    CB_C8=1 CB_NORES=1 timeout -k 10 60 tools/bin/$b winot $shape 10 500 >> $out/cb.txt 2>&1 || { echo "cb $b $shape failed"; tail $out/cb.txt; exit 1; }
  done
done
cat $out/cb.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "variants_bitexact or forward_full or golden or winograd_path or batch_is_per_clip" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
