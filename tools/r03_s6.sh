#!/bin/bash
# round 3: double actor image sets (no act wait before the actor optimiser) -- tests, then bench + anatomy
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03s6}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_schedule_gpu.py \
  tests/test_fused_mlp_gpu.py tests/test_optim_gpu.py tests/test_learner_golden_gpu.py tests/test_agent_gpu.py \
  tests/test_dp_fused_gpu.py tests/test_train_script_gpu.py tests/test_actor_grads_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 2
bash tools/r03_bench_only.sh ${T} || exit 3
