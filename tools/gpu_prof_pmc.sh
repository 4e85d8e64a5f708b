#!/bin/bash
# profile + PMC passes of the weight-streamed kernel on bench_conv C128 k11 (case 3) and k3 (case 1), cfg 21
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_prof.sh "$1" || exit 1
for c in 3 1; do
  bash tools/pmc_conv.sh $c 21 || { echo "pmc failed"; exit 1; }
  python tools/pmc_conv.py pmc_c${c}_g21 conv_wsb > gpurun_out/pmc_c${c}_g21.txt 2>&1
  head -30 gpurun_out/pmc_c${c}_g21.txt
done
