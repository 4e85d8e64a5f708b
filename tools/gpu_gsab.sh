#!/bin/bash
# gather-streamed kernel change: micro-benchmark old vs new, parity tests on the new library, same-box C2 A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-gsab}
TESTS=${2:-"tests/test_gpu_conv_math.py tests/test_gpu_c2_parity.py tests/test_gpu_models.py"}
REPS=${3:-2}
if [ -x build/bench_gs_old ]; then
  timeout -k 10 300 ./build/bench_gs_old 10 1 > gpurun_out/bench_gs_old_$TAG.txt 2>&1 || { echo "bench_gs_old failed"; tail gpurun_out/bench_gs_old_$TAG.txt; exit 1; }
fi
timeout -k 10 300 ./build/bench_gs 10 1 > gpurun_out/bench_gs_new_$TAG.txt 2>&1 || { echo "bench_gs failed"; tail gpurun_out/bench_gs_new_$TAG.txt; exit 1; }
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread $TESTS > gpurun_out/gt_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|^E " gpurun_out/gt_$TAG.log | head -30; exit 1; }
grep -E "passed|failed" gpurun_out/gt_$TAG.log | tail -1
bash tools/ab_lib.sh build/ab/librvcx_base.so $REPS
