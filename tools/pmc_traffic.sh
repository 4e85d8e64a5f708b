# HBM traffic of the C2 step by kernel: two PMC passes (FETCH_SIZE and WRITE_SIZE cannot share one pass),
# counters only (no trace domains), one step after one warm-up. Summarise with tools/pmc_traffic.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$C -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --roofline-pass inline > gpurun_out/pmc_$C.log 2>&1 || exit 1
done
echo pmc done
