#!/bin/bash
# bench_conv checks + the weight-streamed fp16 kernels with / without conv_wsc.hip (RVCX_WSC=0), then the C2 A/B.
cd $GRAFT_REPO_ROOT
timeout -k 5 120 ./build/bench_conv 3 > gpurun_out/bc_checks.txt 2>&1 || { tail -5 gpurun_out/bc_checks.txt; exit 1; }
grep "^check" gpurun_out/bc_checks.txt | grep -c OK; grep "^check" gpurun_out/bc_checks.txt | grep -v OK
grep "^check T=[0-9]* C=[0-9]* N=[0-9]* k=[0-9]* d=[0-9]* cfg=23 (h16" gpurun_out/bc_checks.txt
for c in 0 2 3 4 1; do
  for w in 1 0; do
    echo "WSC=$w $(RVCX_WSC=$w timeout -k 5 60 ./build/bench_conv 20 $c 23)" || exit 1
  done
done
