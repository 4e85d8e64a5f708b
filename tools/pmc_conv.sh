# PMC pass over one conv shape of build/bench_conv (case index, forced cfg); counters in their own run.
CASE=${1:-3}
CFG=${2:-3}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_c${CASE}_g${CFG} -o run -- ./build/bench_conv 5 $CASE $CFG > gpurun_out/pmc_c${CASE}_g${CFG}.log 2>&1
