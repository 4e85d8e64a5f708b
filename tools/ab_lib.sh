# Same-box A/B of two librvcx builds on the C2 bench (RVCX_LIB selects the library).
# usage: bash tools/ab_lib.sh build/ab/librvcx_OLD.so [reps]
OLD=$1
REPS=${2:-3}
for rep in $(seq 1 $REPS); do
  for lib in "$OLD" retrieval-based-voice-conversion-mlx_amd/rvcx/librvcx.so; do
    RVCX_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1
    echo "$(basename $lib) $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])' 2>&1 | tail -1)"
  done
done
