#!/bin/bash
# GPU parity tests: tools/gpu_tests_only.sh TAG [pytest args / test paths; default: tests -m gpu]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-t}; shift
[ $# -eq 0 ] && set -- tests
timeout -k 10 900 python -u -m pytest -m gpu -x -v -s --timeout 120 --timeout-method thread "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|^C[24] |passed|failed|^E " gpurun_out/gpu_tests_$TAG.log | tail -40
exit $rc
