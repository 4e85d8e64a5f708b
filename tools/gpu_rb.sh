set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resblock_fused.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rb_tests.log 2>&1 || { echo "rb tests failed"; tail -40 gpurun_out/rb_tests.log; exit 1; }
tail -3 gpurun_out/rb_tests.log
timeout -k 10 300 python -u tools/bench_rb.py 20 > gpurun_out/bench_rb.txt 2>&1 || { echo "bench_rb failed"; tail -20 gpurun_out/bench_rb.txt; exit 1; }
cat gpurun_out/bench_rb.txt
for v in 1 0 1 0; do RVCX_NO_RBFUSE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab_rb_$v.json 2>gpurun_out/ab_rb.err || { echo "bench failed"; tail -20 gpurun_out/ab_rb.err; exit 1; }; echo "NO_RBFUSE=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_rb_$v.json'));print(d['ms_per_step'], d['roofline']['achieved'])")"; done
