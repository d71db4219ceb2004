#!/bin/bash
# Fused critic leaving 8 / 16 / 32 CUs to the rollout stream vs all CUs: bench AC-IQN + IQN lines, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ASVRL_LIB=variants/libasvrl_res16.so timeout -k 10 300 python -u -m pytest tests/test_critic_fused_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/res_tests.log 2>&1
rc=$?; tail -1 gpurun_out/res_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/sum_ab.sh default res8 res16 res32
