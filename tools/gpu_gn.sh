#!/bin/bash
# parity subset + same-box A/B of the working library against build/ab/librvcx_head.so (the last commit) + kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-gn}
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_c2_parity.py tests/test_gpu_sizes.py > gpurun_out/gt_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gt_$TAG.log; exit 1; }
tail -1 gpurun_out/gt_$TAG.log
bash tools/ab_lib.sh build/ab/librvcx_head.so 3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_$TAG -name "*.db" | head -1)
python tools/prof_summary.py "$DB" 7 > gpurun_out/kstats_$TAG.txt 2>&1
python tools/timeline.py "$DB" 2 > gpurun_out/timeline_$TAG.txt 2>&1
head -4 gpurun_out/timeline_$TAG.txt
