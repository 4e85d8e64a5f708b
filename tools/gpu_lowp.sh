#!/bin/bash
# the reduced-precision generator opt-in: stream tests (fp32 fixture gate), C2 parity subset, C5 fp32 vs bf16 benches,
# C2 A/B against build/ab/librvcx_head.so (the fp32 path must not move)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-lp}
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_stream_ref.py tests/test_gpu_stream.py tests/test_gpu_c2_parity.py tests/test_gpu_models.py > gpurun_out/gt_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gt_$TAG.log; exit 1; }
grep -E "generator bf16|passed|failed" gpurun_out/gt_$TAG.log | tail -3
for p in fp32 bf16; do
  timeout -k 10 300 python -u bench.py --config c5 --gen-precision $p --no-cpu-baseline > gpurun_out/bench_${TAG}_c5_$p.json 2> gpurun_out/bench_${TAG}_c5_$p.err || { echo "c5 $p failed"; tail -5 gpurun_out/bench_${TAG}_c5_$p.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_c5_$p.json').read().strip().splitlines()[-1]); print('c5 $p', d['value'], d['latency_ms'])"
done
bash tools/ab_lib.sh build/ab/librvcx_head.so 2 || exit 1
