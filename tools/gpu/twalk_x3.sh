#!/bin/bash
# conv_twalk_x3 (fp32 split-bf16 frame walk) vs conv_winot5 on the fp32 64-channel temporal convs
# (convbench, 30 clips, 8-channel-blocked input as in the engine), the fp32 tests that cover it, and a
# fp32 bench A/B (A = variant no_twalk_x3, B = product)
out=${1:-gpurun_out/twalk_x3}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
export CB_C8=1
for res in 1 0; do
  if [ $res = 1 ]; then export CB_NORES=1; else unset CB_NORES; fi
  for shp in "30 32 56 56 144 64" "30 32 56 56 48 64"; do
    timeout -k 10 120 $CB winot $shp 10 500 1300 >> $out/cb.txt 2>&1 || { echo "cb $shp failed"; tail $out/cb.txt; exit 1; }
  done
done
cat $out/cb.txt
unset CB_NORES CB_C8
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "twalk_x3 or c8 or per_clip_exact or variants_bitexact or winograd_path" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -60 $out/pytest.log | cut -c1-400; exit 1; }
tail -2 $out/pytest.log
DTYPE=fp32 bash tools/gpu/ab_bf16.sh $out "CLASFV_NO_TWALK_X3=1" ""
