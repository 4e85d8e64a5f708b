#!/bin/bash
# study pass: bench_conv table (all tiles) + per-launch conv dump of C2 steps (inline events, one stream)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-st}
timeout -k 10 400 ./build/bench_conv 20 > gpurun_out/bench_conv_$TAG.txt 2>&1 || { echo "bench_conv failed"; tail gpurun_out/bench_conv_$TAG.txt; exit 1; }
grep -c OK gpurun_out/bench_conv_$TAG.txt; grep FAIL gpurun_out/bench_conv_$TAG.txt
rm -f gpurun_out/convdump_$TAG.csv
RVCX_PROF_DUMP=gpurun_out/convdump_$TAG.csv timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --roofline-pass after > gpurun_out/dump_$TAG.json 2> gpurun_out/dump_$TAG.err || { echo "dump failed"; tail gpurun_out/dump_$TAG.err; exit 1; }
python tools/convdump_summary.py gpurun_out/convdump_$TAG.csv 60 > gpurun_out/convdump_$TAG.txt
head -5 gpurun_out/convdump_$TAG.txt
