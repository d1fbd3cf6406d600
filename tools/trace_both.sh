#!/bin/bash
# kernel traces of the fp32 and bf16 bench runs + per-dispatch summaries (run on the GPU box)
out=$1; mkdir -p $out; export TMPDIR=/tmp
for dt in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace -T -d $out/$dt -o t -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --dtype $dt --extra-bf16 0 > $out/$dt.log 2>&1 || exit 1
  python3 tools/prof_summary.py $out/$dt/t_results.db > $out/$dt.summary.txt || exit 1
done
