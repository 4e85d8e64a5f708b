
timeout -k 10 300 ./build/bench_conv 10 > gpurun_out/bench_conv.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1 || true
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for pol in "1 3" "6 3" "3 3" "6 6"; do
  set -- $pol
  RVCX_CFG_LONG=$1 RVCX_CFG_SHORT=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --roofline-pass inline > gpurun_out/ab.log 2>&1
  echo "long=$1 short=$2 $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])')"
done
done
