# same-box timing of the fused ResBlock pair across library builds (tools/bench_rb.py --one, two-plane fp16: cfg 16)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for lib in $LIBS; do
  for sh in "744000 32 7 1" "744000 32 7 5" "744000 32 11 1" "744000 32 11 5" "744000 32 3 3"; do
    r=$(RVCX_LIB=$lib timeout -k 10 120 python3 tools/bench_rb.py --one $sh 16 20 2>/dev/null | tail -1) || { echo "fail $lib $sh"; exit 1; }
    echo "$lib $r"
  done
done
done
