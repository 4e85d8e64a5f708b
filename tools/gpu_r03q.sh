#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_conv_math.py tests/test_gpu_c2_parity.py tests/test_gpu_models.py tests/test_gpu_resblock_fused.py tests/test_gpu_sizes.py > gpurun_out/gt_q.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|^E " gpurun_out/gt_q.log | head -30; exit 1; }
grep -E "passed|failed" gpurun_out/gt_q.log | tail -1
bash tools/ab_lib.sh build/ab/librvcx_base.so 2 || exit 1
for sh in 0 3 4; do bash tools/pmc_gs.sh $sh q || exit 1; done
