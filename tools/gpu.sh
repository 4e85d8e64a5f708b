#!/bin/bash
# One parameterised GPU-box driver for every measurement this repo takes (run through gpurun):
#   bash tools/gpu.sh TAG STEP [STEP ...]
# Steps run in order; each has its own time limit and the script stops at the first failure.
#   tests[=PATHS]     pytest -m gpu (default: tests/), thread-method timeouts
#   smoke             __graft_entry__.smoke()
#   bench[=ARGS]      bench.py (ARGS with ',' for spaces, e.g. bench=--config,c3,--no-cpu-baseline)
#   configs           C3 / C5 / C4 bench lines (no CPU baseline)
#   prof              rocprofv3 --kernel-trace --stats of the C2 bench + timeline + kernel-family table
#   pmc               the three HBM / MFMA PMC passes of one C2 step (tools/pmc_traffic.sh)
#   bc                build/bench_conv table (checks + every tile)
#   bcx=DIR1,DIR2     bench_conv generator shapes with each DIR's librvcx.so after the in-tree one (timing experiments)
#   pmcconv=CASE,CFG  the PMC passes of bench_conv case CASE on tile cfg CFG (tools/pmc_conv.sh + pmc_conv.py)
#   gru               build/bench_gru (BiGRU steps: full, hand-off only, math only)
#   ab=E1;E2;...      same-box A/B of the C2 bench under env settings (',' for spaces inside one setting)
#   ablib=LIB         same-box A/B of the C2 bench: LIB vs the in-tree librvcx.so
set -o pipefail
# RVCX_* developer knobs are honoured only with RVCX_EXPERIMENTAL=1: set per step (ab, gru, ablib), so tests, smoke,
# bench and profiles run exactly as the driver runs them
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:?tag}; shift
O=gpurun_out

c2line() {  # ms_per_step and conv-family kernel ms of the last JSON line of $1
  tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["family"].get("kernel_ms_per_step"))'
}

for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  echo "== $name $arg"
  case $name in
    tests)
      paths=${arg:-tests}
      timeout -k 10 900 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread ${paths//,/ } > $O/gpu_tests_$TAG.log 2>&1
      rc=$?
      grep -E "PASSED|FAILED|ERROR|passed|failed|^E " $O/gpu_tests_$TAG.log | tail -15
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { tail -20 $O/smoke_$TAG.log; exit 1; }
      tail -1 $O/smoke_$TAG.log ;;
    bench)
      timeout -k 10 500 python -u bench.py ${arg//,/ } > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 1; }
      tail -1 $O/bench_$TAG.json | cut -c1-400 ;;
    configs)
      for c in c3 c5 c4; do
        timeout -k 10 500 python -u bench.py --config $c --no-cpu-baseline > $O/bench_${TAG}_$c.json 2> $O/bench_${TAG}_$c.err || { tail -5 $O/bench_${TAG}_$c.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/bench_${TAG}_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['unit'], d['ms_per_step'])"
      done ;;
    prof)
      # 1 warm-up + 3 timed + 3 host-io + 3 roofline-event steps = 10 pipeline calls traced (the summaries divide by 10)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${arg//,/ } > $O/prof_$TAG.log 2>&1 || { tail -20 $O/prof_$TAG.log; exit 1; }
      DB=$(find $O/prof_$TAG -name "*.db" | head -1)
      python3 tools/timeline.py "$DB" 2 -v > $O/timeline_$TAG.txt 2>&1
      python3 tools/prof_summary.py "$DB" 10 > $O/kstats_$TAG.txt 2>&1
      python3 tools/kfamily.py "$DB" 10 > $O/kfamily_$TAG.txt 2>&1
      head -30 $O/kstats_$TAG.txt ;;
    pmc)
      bash tools/pmc_traffic.sh || exit 1
      python3 tools/pmc_traffic.py gpurun_out > $O/pmc_traffic_$TAG.json || exit 1
      python3 tools/pmc_shapes.py gpurun_out 40 > $O/pmc_shapes_$TAG.txt 2>&1
      head -12 $O/pmc_shapes_$TAG.txt ;;
    bc)
      timeout -k 10 400 ./build/bench_conv 20 ${arg//,/ } > $O/bench_conv_$TAG.txt 2>&1 || { tail $O/bench_conv_$TAG.txt; exit 1; }
      cat $O/bench_conv_$TAG.txt ;;
    bcx)
      # bench_conv on selected generator shapes against alternative library builds (timing-only experiments):
      # bcx=DIR1,DIR2 runs each DIR's librvcx.so (LD_LIBRARY_PATH) after the in-tree one
      for lib in "" ${arg//,/ }; do
        for cc in "1 27" "17 27" "2 23" "3 23" "4 23" "0 23"; do
          r=$(LD_LIBRARY_PATH=$lib timeout -k 10 60 ./build/bench_conv 40 $cc) || { echo "bench_conv $lib $cc failed"; exit 1; }
          echo "lib=${lib:-tree} case/cfg=$cc $r"
        done
      done ;;
    pmcconv)
      bash tools/pmc_conv.sh ${arg%%,*} ${arg##*,} || exit 1
      python3 tools/pmc_conv.py pmc_c${arg%%,*}_g${arg##*,} > $O/pmcconv_${TAG}_${arg%%,*}_${arg##*,}.txt 2>&1
      cat $O/pmcconv_${TAG}_${arg%%,*}_${arg##*,}.txt ;;
    gru)
      for m in 0 1 2 0 1 2; do
        r=$(RVCX_EXPERIMENTAL=1 RVCX_GRU_MODE=$m timeout -k 10 60 ./build/bench_gru 1568 1 10) || { echo "bench_gru mode $m failed"; exit 1; }
        echo "RVCX_GRU_MODE=$m $r"
      done ;;
    ab)
      IFS=';' read -ra envs <<< "X=0;$arg"
      for rep in 1 2; do
        for e in "${envs[@]}"; do
          env RVCX_EXPERIMENTAL=1 ${e//,/ } timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ab_$TAG.log 2>&1 || { echo "bench failed $e"; tail -5 $O/ab_$TAG.log; exit 1; }
          echo "$e $(c2line $O/ab_$TAG.log)"
        done
      done ;;
    ablib)
      for rep in 1 2 3; do
        for lib in "$arg" retrieval-based-voice-conversion-mlx_amd/rvcx/librvcx.so; do
          RVCX_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ab_$TAG.log 2>&1 || { echo "bench failed $lib"; tail -5 $O/ab_$TAG.log; exit 1; }
          echo "$lib $(c2line $O/ab_$TAG.log)"
        done
      done ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "== done"
