#!/bin/bash
# Submit one gpurun call; while the pool has no free slot (gpurun exit 3: nothing ran, nothing charged) wait and
# submit the same call again, at most 20 times. Any other exit (success, a failed or timed-out GPU step, a refusal)
# ends it: a GPU step that ran is never repeated here.
#   bash tools/gpurun_wait.sh OUTFILE TIMEOUT_S 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "busy\|no box\|transient" "$out" || exit $rc
  sleep 100
done
exit 3
