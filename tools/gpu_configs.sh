#!/bin/bash
# parity subset touching the attention / U-Net / generator, then the C3 / C4 / C5 benches (one JSON line each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-cfg}
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_c2_parity.py tests/test_gpu_sizes.py tests/test_gpu_stream_ref.py > gpurun_out/gt_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gt_$TAG.log; exit 1; }
tail -1 gpurun_out/gt_$TAG.log
for c in c3 c5 c4; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${TAG}_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['unit'], d['ms_per_step'], d.get('config',{}).get('workload',''))"
done
