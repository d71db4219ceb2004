#!/bin/bash
# the pipelined-learner test under both encoder modes (stops at the first failure), then the partial-sum A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for E in 0 1; do
  ASVRL_ENC_IN_KERNEL=$E timeout -k 10 300 python -u -m pytest tests/test_learn_kernels_gpu.py -k "pipelined_target" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pipe_enc$E.log 2>&1
  rc=$?; echo "enc=$E rc=$rc"; grep -E "PASSED|FAILED|Fatal|passed|failed" gpurun_out/pipe_enc$E.log | head -5; [ $rc -eq 0 ] || exit $rc
done
bash tools/sum_ab.sh default sacc16 sacc32 swav16
