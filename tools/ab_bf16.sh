#!/bin/bash
# kernel trace of the bf16 headline run
out=$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $out/t -o t -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --dtype bf16 --extra-bf16 0 > $out/run.log 2>&1
