#!/bin/bash
# tests subset + same-box A/B (base vs new) + rocprofv3 kernel trace of the C2 bench with a step timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-t}; shift
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_conv_math.py tests/test_gpu_c2_parity.py tests/test_gpu_models.py tests/test_gpu_resblock_fused.py tests/test_gpu_sizes.py tests/test_gpu_vocoders.py tests/test_gpu_nof0.py > gpurun_out/gt_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|^E " gpurun_out/gt_$TAG.log | head -30; exit 1; }
grep -E "passed|failed" gpurun_out/gt_$TAG.log | tail -1
bash tools/ab_lib.sh build/ab/librvcx_base.so 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_$TAG -name "*.db" | head -1)
python tools/timeline.py "$DB" 2 > gpurun_out/timeline_$TAG.txt 2>&1
python tools/prof_summary.py "$DB" 7 > gpurun_out/kstats_$TAG.txt 2>&1
head -5 gpurun_out/timeline_$TAG.txt; head -25 gpurun_out/kstats_$TAG.txt
