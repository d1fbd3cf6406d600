#!/bin/bash
# Profiles of the bench workload (run on the GPU box): kernel trace + stats and HBM traffic passes
# (FETCH_SIZE and WRITE_SIZE each in a pass of its own), fp32 and bf16 headline runs.
# usage: bash tools/gpu_profile.sh OUTDIR
out=${1:-gpurun_out/prof}; mkdir -p $out; export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0"
for dt in fp32 bf16; do
  mkdir -p $out/$dt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -T -d $out/$dt/trace -o t -- python3 $B --dtype $dt > $out/$dt/trace.log 2>&1 || { echo "trace $dt failed"; tail -20 $out/$dt/trace.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -T -d $out/$dt/$c -o p -- python3 $B --dtype $dt > $out/$dt/$c.log 2>&1 || { echo "pmc $c $dt failed"; tail -20 $out/$dt/$c.log; exit 1; }
  done
  python3 tools/prof_summary.py $(find $out/$dt/trace -name 't_results.db' | head -1) $(find $out/$dt/FETCH_SIZE -name 'p_results.db' | head -1) $(find $out/$dt/WRITE_SIZE -name 'p_results.db' | head -1) > $out/$dt/summary.txt || exit 1
  find $out/$dt/trace -name 't_kernel_stats.csv' -exec cp {} $out/$dt/kernel_stats.csv \;
done
