#!/bin/bash
# bench_conv table (checks + every tile) then a same-box env A/B of the C2 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-bc}; shift
timeout -k 10 400 ./build/bench_conv 20 > gpurun_out/bench_conv_$TAG.txt 2>&1 || { echo "bench_conv failed"; tail gpurun_out/bench_conv_$TAG.txt; exit 1; }
grep -E "^check cfg=2[3-9]" gpurun_out/bench_conv_$TAG.txt
grep -v "^check" gpurun_out/bench_conv_$TAG.txt | grep gen | sed -E 's/ [ef](1[0-6]|2[0-2]|-1|1|3)p?: *[0-9.]+\*?//g'
for rep in 1 2; do
  for e in X=0 "$@"; do
    env $e timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abb_$TAG.log 2>&1 || { echo "bench failed $e"; tail -5 gpurun_out/abb_$TAG.log; exit 1; }
    echo "$e $(tail -1 gpurun_out/abb_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])')"
  done
done
