#!/bin/bash
out=${1:-gpurun_out/w4st}; mkdir -p $out; export TMPDIR=/tmp
cb=tools/bin/convbench
{ timeout -k 10 200 $cb wino4 30 32 56 56 64 144 20 0 128 4096 4 0 4096; } > $out/st.txt 2>&1 || { echo "st failed"; cat $out/st.txt; exit 1; }
cat $out/st.txt
