#!/bin/bash
# round 3: the replay/learn kernel tests, then the PMC passes of tools/pmc_run.sh on the bench workload
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_learn_kernels_gpu.py tests/test_fused_critic_gpu.py tests/test_critic_fused_gpu.py tests/test_learner_golden_gpu.py tests/test_fused_iqn_gpu.py tests/test_iqn_fused_gpu.py > gpurun_out/${T}_pytest.log 2>&1 || exit 2
rm -rf gpurun_out/pmc
BENCH_ARGS="--steps 10 --warmup 5 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0" PMC_EXTRA=1 timeout -k 10 1200 bash tools/pmc_run.sh || exit 3
python tools/pmc_summary.py gpurun_out/pmc --json gpurun_out/${T}_pmc_summary.json > gpurun_out/${T}_pmc_summary.txt 2>&1
