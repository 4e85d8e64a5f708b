# Same-box A/B of env settings on the C2 bench. usage: bash tools/ab_env.sh REPS "VAR=a" "VAR=b" ...
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1
    echo "$setting $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])' 2>&1 | tail -1)"
  done
done
