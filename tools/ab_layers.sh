#!/bin/bash
# A/B the conv tile configurations: one kernel-trace run per env setting, per-layer summary.
# usage (on the GPU box): bash tools/ab_layers.sh OUTDIR "ENV1" "ENV2" ...
out=$1; shift
export TMPDIR=/tmp
mkdir -p $out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace -T -d $out/cfg$i -o t -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $out/cfg$i.log 2>&1 || exit 1
  echo "== cfg$i: $cfg" >> $out/summary.txt
  tail -1 $out/cfg$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'fwd_ms_per_clip', d['roofline']['forward_ms_per_clip'], 'frac', d['roofline']['frac'])" >> $out/summary.txt
  python3 tools/prof_summary.py $out/cfg$i/t_results.db | sed -n '/per-dispatch/,$p' >> $out/summary.txt
done
