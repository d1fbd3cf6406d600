set -e
export TMPDIR=/tmp
bash tools/convbench.sh build
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
for ko in 0 4; do
  CB_NORES=1 timeout -s KILL 60 rocprofv3 --pmc $C -d gpurun_out/pq$ko -o p --output-format csv -- gpurun_out/convbench winoq 30 32 56 56 64 144 3 $ko > gpurun_out/pq$ko.log 2>&1
done
