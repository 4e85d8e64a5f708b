#!/bin/bash
# same-box A/B of env variants on the current library (no tests) + rocprofv3 kernel trace of the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-x}; shift
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abx_$TAG.log 2>&1 || { echo "bench failed $*"; tail -5 gpurun_out/abx_$TAG.log; return 1; }
  echo "$* $(tail -1 gpurun_out/abx_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])')"
}
for rep in 1 2; do
  for e in X=0 "$@"; do run $e || exit 1; done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_$TAG -name "*.db" | head -1)
python tools/timeline.py "$DB" 2 > gpurun_out/timeline_$TAG.txt 2>&1
python tools/prof_summary.py "$DB" 7 > gpurun_out/kstats_$TAG.txt 2>&1
head -4 gpurun_out/timeline_$TAG.txt
