#!/bin/bash
# kernel + HIP API trace of the C2 bench (no counters), CSV, summarised on the box (the trace itself is large)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d /tmp/prof_ht -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ht.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_ht.log; exit 1; }
python3 tools/launch_gaps.py /tmp/prof_ht 2 > gpurun_out/launch_gaps.txt 2>&1
python3 tools/launch_gaps.py /tmp/prof_ht 3 >> gpurun_out/launch_gaps.txt 2>&1
tail -40 gpurun_out/launch_gaps.txt
