# Marginal wall cost of trivial launches inserted into the C2 step (measurement library build/exx, built with
# -DRVCX_EXP_EXTRA): RVCX_EXTRA launches per TextEncoder layer (6 layers) or, with RVCX_EXTRA_AT=gen, before each
# generator ResBlock (12); RVCX_NO_OVERLAP=1 (with RVCX_EXPERIMENTAL=1) runs the step on one stream
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {
  env RVCX_LIB=build/exx/librvcx.so "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/extra.log 2>&1 || { tail -5 gpurun_out/extra.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/extra.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for rep in 1 2; do
  run RVCX_EXTRA=0
  run RVCX_EXTRA=32
  run RVCX_EXTRA=16 RVCX_EXTRA_AT=gen
  run RVCX_EXPERIMENTAL=1 RVCX_NO_OVERLAP=1 RVCX_EXTRA=0
  run RVCX_EXPERIMENTAL=1 RVCX_NO_OVERLAP=1 RVCX_EXTRA=32
done
