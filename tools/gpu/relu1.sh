#!/bin/bash
# one-instruction ReLU / packed subtraction / lean wino4w epilogue: full GPU tests, convbench of the
# affected kernels, fp32 kernel trace. usage (GPU box): bash tools/gpu/relu1.sh OUTDIR
out=${1:-gpurun_out/relu1}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "tests failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
CB=tools/bin/convbench
for shape in "30 32 56 56 64 144" "30 16 28 28 128 288" "30 8 14 14 256 576"; do
  timeout -k 10 60 $CB wino4w $shape 10 0 256 >> $out/cb.txt 2>&1 || { echo "cb failed"; exit 1; }
done
CB_C8=1 timeout -k 10 60 $CB winot 30 32 56 56 144 64 10 500 >> $out/cb.txt 2>&1 || { echo "cb failed"; exit 1; }
cat $out/cb.txt
bash tools/gpu/trace.sh $out/trace > /dev/null && grep -E "^conv|^decoder|forward GPU" $out/trace/summary.txt | head -12
