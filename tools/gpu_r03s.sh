#!/bin/bash
# tests subset + same-box A/B (base lib, new lib, new lib with env variants) + per-launch conv dump
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-s}; shift
[ -x build/bench_gs ] && timeout -k 10 300 ./build/bench_gs 10 1 > gpurun_out/bench_gs_$TAG.txt 2>&1
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_conv_math.py tests/test_gpu_c2_parity.py tests/test_gpu_models.py tests/test_gpu_resblock_fused.py tests/test_gpu_sizes.py > gpurun_out/gt_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|^E " gpurun_out/gt_$TAG.log | head -30; exit 1; }
grep -E "passed|failed" gpurun_out/gt_$TAG.log | tail -1
run() {  # run LIB ENV...
  local lib=$1; shift
  env "$@" RVCX_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$TAG.log 2>&1 || { echo "bench failed $lib $*"; tail -5 gpurun_out/ab_$TAG.log; return 1; }
  echo "$(basename $lib) $* $(tail -1 gpurun_out/ab_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])')"
}
NEW=retrieval-based-voice-conversion-mlx_amd/rvcx/librvcx.so
for rep in 1 2; do
  run build/ab/librvcx_base.so X=0 || exit 1
  for e in "X=0" "$@"; do run $NEW $e || exit 1; done
done
rm -f gpurun_out/convdump_$TAG.csv
RVCX_PROF_DUMP=gpurun_out/convdump_$TAG.csv timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --roofline-pass after > gpurun_out/dump_$TAG.json 2> gpurun_out/dump_$TAG.err || { echo "dump failed"; tail gpurun_out/dump_$TAG.err; exit 1; }
python tools/convdump_summary.py gpurun_out/convdump_$TAG.csv 40 > gpurun_out/convdump_$TAG.txt
head -30 gpurun_out/convdump_$TAG.txt
