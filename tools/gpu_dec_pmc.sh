#!/bin/bash
# Decoder (30 clips, 32x112x112) SQ counter passes: where the wave cycles go (issue vs waits vs MFMA).
# One rocprofv3 --pmc pass per counter set (<= 8 SQ counters each), each under its own time limit.
out=gpurun_out/dec_pmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 5 60 rocprofv3 -L > $R/$out/counters.txt 2>&1 || exit 1
have() { for c in "$@"; do grep -qw "$c" $R/$out/counters.txt || { echo "missing counter $c"; return 1; }; done; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAVES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  have $P || continue
  timeout -s KILL 90 rocprofv3 --pmc $P -d $R/$out/p$i -o p$i --output-format csv -- $R/tools/bin/convbench dec 30 32 112 112 5 0 > $R/$out/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$R/$out" <<'EOF'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "decoder_kernel" not in r["Kernel_Name"]: continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
with open(out + "/summary.txt", "w") as fo:
    for k in sorted(tot):
        line = f"{k:32s} total {tot[k]:.4g} over {n[k]} records"
        print(line); fo.write(line + "\n")
EOF
