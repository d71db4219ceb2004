#!/bin/bash
# round 3: learner-alone A/B (one-launch reduction + Adam vs two launches), its kernel stats, then the
# reduce+Adam bit-identity test
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03}
timeout -k 10 300 python -u tools/bench_learn.py > gpurun_out/${T}_learn_ab.txt 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/${T}_learn_prof && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_learn_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_learn.py --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/${T}_learn_prof.txt 2>&1 || exit 3
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_critic_gpu.py tests/test_critic_fused_gpu.py tests/test_fused_iqn_gpu.py tests/test_iqn_fused_gpu.py tests/test_learner_golden_gpu.py > gpurun_out/${T}_learn_test.log 2>&1
