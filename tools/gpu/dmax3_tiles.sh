#!/bin/bash
# conv_dma_x3 tile-shape sweep (CB_X3CFG "MT NT S", CB_X3WN) on the forward's largest strided / layer4
# convs. usage (GPU box): bash tools/gpu/dmax3_tiles.sh OUTDIR
out=${1:-gpurun_out/dmax3_tiles}; mkdir -p $out; export TMPDIR=/tmp
CB=tools/bin/convbench
run() {  # label env... -- args
  echo "== $*" >> $out/cb.txt
  env "$@" timeout -k 10 60 $CB $SHAPE 10 710 >> $out/cb.txt 2>&1 || { echo "failed: $*"; tail -5 $out/cb.txt; exit 1; }
}
SHAPE="sp 30 32 56 56 64 240"
for c in "2 5 2" "1 5 2" "4 5 2" "2 5 3" "2 3 2"; do run CB_STRIDE=2 CB_NORES=1 CB_X3CFG="$c"; done
SHAPE="tp 30 32 28 28 240 128"
for c in "2 8 2" "1 8 2" "4 8 2" "4 4 2" "2 4 2" "2 4 3"; do run CB_STRIDE=2 CB_NORES=1 CB_X3CFG="$c"; done
run CB_STRIDE=2 CB_NORES=1 CB_X3CFG="2 8 2" CB_X3WN=2
SHAPE="sp 30 16 28 28 128 480"
for c in "2 6 2" "1 6 2" "4 6 2" "2 6 3" "1 6 3" "2 5 2" "4 5 2"; do run CB_STRIDE=2 CB_NORES=1 CB_X3CFG="$c"; done
SHAPE="sp 30 4 7 7 512 1152"
for c in "2 8 2" "1 8 2" "4 8 2" "2 6 2" "1 6 2"; do run CB_NORES=1 CB_X3CFG="$c"; done
grep -E "^==|ko=" $out/cb.txt
