#!/bin/bash
# round 3: the pipelined AC-IQN schedule -- schedule / learner tests, the default bench, one step's anatomy
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03s5}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_schedule_gpu.py \
  tests/test_learn_kernels_gpu.py tests/test_learner_golden_gpu.py tests/test_agent_gpu.py tests/test_dp_fused_gpu.py \
  tests/test_train_script_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 2
TESTS=tests/test_actor_grads_gpu.py bash tools/r03_bench_anatomy.sh ${T} || exit 3
