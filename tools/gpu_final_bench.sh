#!/bin/bash
# the headline bench (with the CPU baseline and roofline.traffic from profiles/pmc_traffic.json) + C3 / C4 lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-fb}
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
tail -1 gpurun_out/bench_$TAG.json | cut -c1-300
for c in c3 c4; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'])"
done
