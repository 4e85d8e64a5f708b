#!/bin/bash
# BiGRU hand-off variants: bench_gru per RVCX_GRU_FLAGS value, then the C2 same-box A/B with the variants
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for f in 0 1 2 3 0 1 2 3; do
  echo "flags=$f $(RVCX_GRU_FLAGS=$f timeout -k 10 60 ./build/bench_gru 1568 1 10)" || exit 1
done
for f in 1 3; do
  RVCX_GRU_FLAGS=$f timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_c2_parity.py > gpurun_out/gt_gru$f.log 2>&1 || { echo "tests failed flags=$f"; tail -20 gpurun_out/gt_gru$f.log; exit 1; }
  echo "flags=$f $(tail -1 gpurun_out/gt_gru$f.log)"
done
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abg.log 2>&1 || { echo "bench failed $*"; tail -5 gpurun_out/abg.log; return 1; }
  echo "$* $(tail -1 gpurun_out/abg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])')"
}
for rep in 1 2; do
  for e in RVCX_GRU_FLAGS=0 RVCX_GRU_FLAGS=1 RVCX_GRU_FLAGS=3 "RVCX_GRU_FLAGS=1 RVCX_HUBERT_GATE=1" "RVCX_GRU_FLAGS=1 RVCX_HUBERT_GATE=3"; do run $e || exit 1; done
done
