#!/bin/bash
# same-box A/B of env variants (C2 bench, 2 reps each) + a rocprofv3 kernel trace per variant with the step timeline
# usage: bash tools/gpu_envprof.sh TAG VAR=VAL [VAR=VAL ...]   (X=0 is the default variant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-e}; shift
run() {
  env $@ timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abe_$TAG.log 2>&1 || { echo "bench failed $*"; tail -5 gpurun_out/abe_$TAG.log; return 1; }
  echo "$* $(tail -1 gpurun_out/abe_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])')"
}
for rep in 1 2; do
  for e in X=0 "$@"; do run $e || exit 1; done
done
i=0
for e in X=0 "$@"; do
  i=$((i + 1))
  for kv in $e; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}_$i.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_${TAG}_$i.log; exit 1; }
  for kv in $e; do unset "${kv%%=*}"; done
  DB=$(find gpurun_out/prof_${TAG}_$i -name "*.db" | head -1)
  python tools/timeline.py "$DB" 2 -v > gpurun_out/timeline_${TAG}_$i.txt 2>&1
  python tools/prof_summary.py "$DB" 7 > gpurun_out/kstats_${TAG}_$i.txt 2>&1
  echo "== $e"; head -3 gpurun_out/timeline_${TAG}_$i.txt
  python3 tools/kfamily.py "$DB"
done
