#!/bin/bash
# config[3] forwards with 2 vs 1 in flight (A B A B)
out=${1:-gpurun_out/c3_inflight}; mkdir -p $out; export TMPDIR=/tmp
for k in 2 1 2 1; do
timeout -k 10 300 python -u bench.py --workload c3 --steps 6 --warmup 2 --inflight $k > $out/c3_$k.log 2>&1 || { echo "c3 failed"; tail -30 $out/c3_$k.log; exit 1; }
echo -n "inflight $k "; tail -1 $out/c3_$k.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
