#!/bin/bash
# round 3: 16-byte partial sums -- the reduction / learner tests, then bench + anatomy
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03s7}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_wgrad_gpu.py \
  tests/test_learner_golden_gpu.py tests/test_chain_schedule_gpu.py tests/test_critic_fused_gpu.py \
  tests/test_iqn_fused_gpu.py tests/test_fused_rainbow_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 2
bash tools/r03_bench_only.sh ${T} || exit 3
