#!/bin/bash
# Head run (suite, bench, kernel stats, PMC) at the read-ahead default, then the dWc read-ahead A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash tools/head_run2.sh > gpurun_out/head_run2.out 2>&1 || { tail -20 gpurun_out/head_run2.out; exit 1; }
tail -2 gpurun_out/head_run2.out | cut -c1-200
cd $R && ASVRL_LIB=variants/libasvrl_dwc1.so timeout -k 10 300 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/dwc_tests.log 2>&1
rc=$?; tail -1 gpurun_out/dwc_tests.log; [ $rc -eq 0 ] || exit $rc
for L in dwc0 dwc1 dwc0 dwc1 dwc0 dwc1; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 120 python tools/fused_time.py >> gpurun_out/dwc_time.jsonl 2>gpurun_out/dwc_time.err || exit 1
done
cat gpurun_out/dwc_time.jsonl
bash tools/sum_ab.sh dwc0 dwc1
