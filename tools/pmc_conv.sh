# PMC passes over one conv shape of build/bench_conv (case index, forced cfg: every arithmetic of that tile runs);
# each counter set in its own rocprofv3 run; summarise with tools/pmc_conv.py pmc_c<CASE>_g<CFG>
CASE=${1:-3}
CFG=${2:-23}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_SALU"
P3="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES SQ_WAVES SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_c${CASE}_g${CFG}_p$i -o run -- ./build/bench_conv 5 $CASE $CFG > gpurun_out/pmc_c${CASE}_g${CFG}_p$i.log 2>&1 || exit 1
done
