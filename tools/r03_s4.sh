#!/bin/bash
# round 3: learner-chain tests, actor-gradient phase stamps, default bench + one step's anatomy
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03s4}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_actor_grads_gpu.py \
  tests/test_optim_gpu.py tests/test_learner_golden_gpu.py tests/test_agent_gpu.py tests/test_chain_schedule_gpu.py \
  tests/test_dp_fused_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 2
bash tools/r03_ag_stamps.sh ${T} || exit 3
TESTS=tests/test_smoke_gpu.py bash tools/r03_bench_anatomy.sh ${T} || exit 4
