#!/bin/bash
# same-box A/B of bench_conv binaries: tools/gpu_ab_conv.sh TAG BIN1 BIN2 ... (each run twice, interleaved)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  for b in "$@"; do
    timeout -k 10 240 ./build/$b 20 > gpurun_out/abc_${TAG}_${b}_$rep.txt 2>&1 || { echo "$b failed"; tail -5 gpurun_out/abc_${TAG}_${b}_$rep.txt; exit 1; }
    echo "== $b rep $rep"; grep -v "^check" gpurun_out/abc_${TAG}_${b}_$rep.txt | grep "gen\." | sed 's/  */ /g' | cut -c1-60,120-200
  done
done
