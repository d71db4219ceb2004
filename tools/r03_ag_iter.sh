#!/bin/bash
# round 3: actor-gradient kernel iteration -- its tests, then the phase stamps with and without the optimiser
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03ag}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_actor_grads_gpu.py \
  > gpurun_out/${T}_pytest.log 2>&1 || exit 2
bash tools/r03_ag_stamps.sh ${T} || exit 3
