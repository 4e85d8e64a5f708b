#!/bin/bash
# bench_conv table + PMC passes of the weight-streamed kernel (cfg 21) on C128 k11 (case 3) and k3 (case 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-cs}
timeout -k 10 300 ./build/bench_conv 20 > gpurun_out/bench_conv_$TAG.txt 2>&1 || { echo "bench_conv failed"; tail gpurun_out/bench_conv_$TAG.txt; exit 1; }
grep -v "^check" gpurun_out/bench_conv_$TAG.txt | grep gen
for c in 3 1; do
  bash tools/pmc_conv.sh $c 21 || { echo "pmc failed"; exit 1; }
  python tools/pmc_conv.py pmc_c${c}_g21 conv_wsb > gpurun_out/pmc_c${c}_g21.txt 2>&1
done
