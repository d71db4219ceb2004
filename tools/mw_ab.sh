#!/bin/bash
# Split actor kernels with the chain's weight fragments (mw1) / and LDS operands (mw2) fetched first vs default.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for L in mw1 mw2; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${L}_tests.log 2>&1
  rc=$?; echo $L; tail -1 gpurun_out/${L}_tests.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/sum_ab.sh default mw1 mw2
