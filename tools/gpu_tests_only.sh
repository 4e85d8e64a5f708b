#!/bin/bash
# GPU parity tests only (optionally a -k filter): tools/gpu_tests_only.sh TAG [pytest args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-t}; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|^C[24] |passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -60
exit $rc
