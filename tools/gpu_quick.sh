#!/bin/bash
# quick pass after a kernel change: selected GPU tests, then same-box A/B of bench.py C2 under env settings
# usage: tools/gpu_quick.sh TAG "TESTS" "ENV1" "ENV2" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; TESTS=$2; shift 2
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread $TESTS > gpurun_out/gq_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|^E " gpurun_out/gq_$TAG.log | head -30; exit 1; }
  grep -E "passed|failed" gpurun_out/gq_$TAG.log | tail -2
fi
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/gq_${TAG}_$i.json 2>gpurun_out/gq_${TAG}_$i.err || { echo "bench failed: $e"; tail -20 gpurun_out/gq_${TAG}_$i.err; exit 1; }
    echo "[$e] $(python -c "import json;d=json.load(open('gpurun_out/gq_${TAG}_$i.json'));print(d['ms_per_step'], d['roofline']['achieved'], d['roofline']['kernel_ms_per_step'])")"
  done
done
