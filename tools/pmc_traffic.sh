# HBM traffic and MFMA busy of the C2 step by conv launch: three PMC passes (FETCH_SIZE and WRITE_SIZE cannot share
# one pass; the SQ/GRBM counters get their own), counters only (no trace domains), one timed step after one warm-up
# with the per-launch events inline (single stream: dispatch order = the RVCX_PROF_DUMP line order of the step).
# Summarise with tools/pmc_traffic.py (family totals, profiles/pmc_traffic.json) and tools/pmc_shapes.py (per shape).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=${C%% *}
  rm -f gpurun_out/convdump_$tag.csv
  RVCX_PROF_DUMP=gpurun_out/convdump_$tag.csv timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$tag -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --roofline-pass inline > gpurun_out/pmc_$tag.log 2>&1 || exit 1
done
echo pmc done
