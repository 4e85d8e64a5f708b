#!/bin/bash
# round-3 pass: selected GPU tests, then a rocprofv3 kernel trace of the C2 bench with the critical-path timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r03}; shift
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|^C[24] |passed|failed|Error" gpurun_out/gpu_tests_$TAG.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log
DB=$(find gpurun_out/prof_$TAG -name "*.db" | head -1)
python tools/timeline.py "$DB" 2 > gpurun_out/timeline_$TAG.txt 2>&1; cat gpurun_out/timeline_$TAG.txt | head -40
