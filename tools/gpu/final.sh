#!/bin/bash
# Round-end GPU pass: full GPU tests, smoke, default bench line (config[1] + extras), config[2] bench,
# kernel trace (--stats) and the FETCH_SIZE / WRITE_SIZE PMC passes of the fp32 forward.
# usage (GPU box): bash tools/gpu/final.sh OUTDIR [quick]   (quick: no PMC passes)
out=${1:-gpurun_out/final}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
timeout -k 10 400 python -u bench.py --workload c2 --steps 5 --warmup 2 > $out/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -30 $out/bench_c2.log; exit 1; }
tail -1 $out/bench_c2.log | cut -c1-300
B="bench.py --steps 2 --warmup 1 --cpu-baseline 0 --extra-bf16 0 --extra-c3 0 --extra-stream 0 --parity-random 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -T -d $out/trace -o t -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed"; tail -30 $out/trace.log; exit 1; }
find $out/trace -name 't_kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
if [ "$2" = quick ]; then
  python3 tools/prof_summary.py $(find $out/trace -name 't_results.db' | head -1) > $out/summary.txt
  head -14 $out/summary.txt; exit 0
fi
# FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md): fp32 config[1], bf16 config[4],
# fp32 config[3] (64x224x224 clips)
for tag in fp32 bf16 fp32_c3; do
  case $tag in fp32) A="$B";; bf16) A="$B --dtype bf16";;
    fp32_c3) A="bench.py --workload c3 --steps 2 --warmup 1 --c3-batch 8";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace -T -d $out/trace_$tag -o t -- python3 $A > $out/trace_$tag.log 2>&1 || { echo "trace $tag failed"; tail -30 $out/trace_$tag.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -T -d $out/${c}_$tag -o p -- python3 $A > $out/${c}_$tag.log 2>&1 || { echo "pmc $c $tag failed"; tail -20 $out/${c}_$tag.log; exit 1; }
  done
  python3 tools/prof_summary.py $(find $out/trace_$tag -name 't_results.db' | head -1) $(find $out/FETCH_SIZE_$tag -name 'p_results.db' | head -1) $(find $out/WRITE_SIZE_$tag -name 'p_results.db' | head -1) > $out/summary_$tag.txt
  echo "== $tag"; head -12 $out/summary_$tag.txt; grep "^pmc" $out/summary_$tag.txt
done
