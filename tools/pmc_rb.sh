# PMC passes over the fused ResBlock pair kernel at one shape (tools/bench_rb.py --one T C k d cfg reps); each
# counter set in its own rocprofv3 run; summarise with tools/pmc_conv.py pmc_rb_<tag> k_rb_pair
T=$1; C=$2; K=$3; D=$4; CFG=$5; TAG=${6:-$C_$K}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_MFMA"
P3="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES SQ_WAVES"
P4="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_rb_${TAG}_p$i -o run -- python3 tools/bench_rb.py --one $T $C $K $D $CFG 5 > gpurun_out/pmc_rb_${TAG}_p$i.log 2>&1 || exit 1
done
