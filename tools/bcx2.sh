#!/bin/bash
# bench_conv "case,cfg" pairs on the in-tree library and on each library directory in $LIBS (same box)
for lib in "" $LIBS; do
  for cc in "$@"; do
    r=$(LD_LIBRARY_PATH=$lib timeout -k 10 60 ./build/bench_conv 40 ${cc/,/ }) || { echo "bench_conv $cc failed"; exit 1; }
    echo "lib=${lib:-tree} $cc $r"
  done
done
