#!/bin/bash
# GPU parity subset (conv paths + pipeline) then a same-box env A/B of the C2 bench (2 reps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-abt}; shift
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_math.py tests/test_gpu_split.py tests/test_gpu_models.py tests/test_gpu_c2_parity.py tests/test_gpu_sizes.py tests/test_gpu_resblock_fused.py > gpurun_out/gt_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gt_$TAG.log; exit 1; }
tail -1 gpurun_out/gt_$TAG.log
for rep in 1 2; do
  for e in X=0 "$@"; do
    env $e timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abt_$TAG.log 2>&1 || { echo "bench failed $e"; tail -5 gpurun_out/abt_$TAG.log; exit 1; }
    echo "$e $(tail -1 gpurun_out/abt_$TAG.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])')"
  done
done
