#!/bin/bash
# Kernel traces (--stats) and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) of the fp32
# config[1], bf16 config[4] and fp32 config[3] forwards, then the clock / MFMA-busy pass (clock.sh).
# usage (GPU box): bash tools/gpu/pmc_pass.sh OUTDIR
out=${1:-gpurun_out/pmc}; mkdir -p $out; export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --inflight 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0 --extra-c2-ragged 0"
for tag in fp32 bf16 fp32_c3; do
  case $tag in fp32) A="$B";; bf16) A="$B --dtype bf16";;
    fp32_c3) A="bench.py --workload c3 --steps 2 --warmup 1 --c3-batch 8";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $out/trace_$tag -o t -- python3 $A > $out/trace_$tag.log 2>&1 || { echo "trace $tag failed"; tail -30 $out/trace_$tag.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -T -d $out/${c}_$tag -o p -- python3 $A > $out/${c}_$tag.log 2>&1 || { echo "pmc $c $tag failed"; tail -20 $out/${c}_$tag.log; exit 1; }
  done
  python3 tools/prof_summary.py $(find $out/trace_$tag -name 't_results.db' | head -1) $(find $out/FETCH_SIZE_$tag -name 'p_results.db' | head -1) $(find $out/WRITE_SIZE_$tag -name 'p_results.db' | head -1) > $out/summary_$tag.txt
  echo "== $tag"; head -12 $out/summary_$tag.txt; grep "^pmc" $out/summary_$tag.txt
done
bash tools/gpu/clock.sh $out/clock
