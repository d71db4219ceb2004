#!/bin/bash
# Weight read-ahead in the critic forward / actor / IQN-max kernels (cra1) vs the default: tests on cra1, bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ASVRL_LIB=variants/libasvrl_cra1.so timeout -k 10 400 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_iqn_fused_gpu.py tests/test_learner_golden_gpu.py tests/test_fused_critic_gpu.py tests/test_fused_iqn_gpu.py tests/test_agent_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/cra_tests.log 2>&1
rc=$?; tail -1 gpurun_out/cra_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/sum_ab.sh default cra1
