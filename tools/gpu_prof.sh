#!/bin/bash
# rocprofv3 kernel trace of the C2 bench (3 timed + 3 roofline-event steps after 1 warmup) + critical-path timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-p}; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
grep '^{' gpurun_out/prof_$TAG.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'TF', d['roofline']['achieved'])"
DB=$(find gpurun_out/prof_$TAG -name "*.db" | head -1)
python tools/timeline.py "$DB" 2 > gpurun_out/timeline_$TAG.txt 2>&1
python tools/prof_summary.py "$DB" 7 > gpurun_out/kstats_$TAG.txt 2>&1
head -40 gpurun_out/timeline_$TAG.txt
