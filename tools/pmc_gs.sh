#!/bin/bash
# PMC passes of build/bench_gs on one shape (its split plan only): bash tools/pmc_gs.sh SHAPE [TAG]
SH=${1:-0}; TAG=${2:-g}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVES"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_SCA"
P3="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH"
P4="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcgs_${TAG}_s${SH}_p$i -o run -- ./build/bench_gs 10 0 $SH 1 > gpurun_out/pmcgs_${TAG}_s${SH}_p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcgs_${TAG}_s${SH}_p$i.log; exit 1; }
done
python3 tools/pmc_gs_sum.py gpurun_out pmcgs_${TAG}_s${SH} conv_gs16
