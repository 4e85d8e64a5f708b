# Same-box A/B of bench.py C2 under environment settings: tools/gpu_ab.sh "ENV1" "ENV2" ... (each run twice, interleaved)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab_$i.json 2>gpurun_out/ab_$i.err || { echo "bench failed: $e"; tail -20 gpurun_out/ab_$i.err; exit 1; }
    echo "[$e] $(python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print(d['ms_per_step'], d['roofline']['achieved'], d['roofline']['kernel_ms_per_step'])")"
  done
done
