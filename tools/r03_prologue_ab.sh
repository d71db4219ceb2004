#!/bin/bash
# round 3: the learn prologue with its weight fragments fetched ahead -- its kernel tests, the chain
# tests, the bench (single-wait schedule A/B on the same box), one graph-replayed step's kernels
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_learn_kernels_gpu.py tests/test_chain_schedule_gpu.py tests/test_learner_golden_gpu.py > gpurun_out/${T}_pytest.log 2>&1 || exit 2
O=gpurun_out/${T}_ab.txt
: > $O
run() {
  echo "== $*" >> $O
  env "$@" timeout -k 10 120 python -u bench.py --steps 40 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
    --plateau-envs 0 --no-cpu-baseline 2>> gpurun_out/${T}_ab.err | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" >> $O || return 1
}
for i in 1 2; do
run X=0 && run DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run ASVRL_TMP_ONEWAIT=1 && run ASVRL_TMP_ONEWAIT=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit 3
done
cd /tmp && export TMPDIR=/tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/${T}_prof && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run --output-format csv rocpd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.err || exit 4
cd $GRAFT_REPO_ROOT && python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
exit 0
