#!/bin/bash
# IQN loop: the learner's draw / target pass ahead of the rollout's act (VecTrainer.iqn_head_first 0 / 1 / 2),
# after its bit-identity test; alternating, two reps
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_chain_schedule_gpu.py::test_iqn_learner_head_first_matches_default" > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
ARGS="--steps 10 --warmup 10 --iqn-steps 300 --no-cpu-baseline --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2; do for H in 0 1 2; do
  printf "%s head=%s " $rep $H >> gpurun_out/${T}_ab.txt
  timeout -k 10 200 python bench.py $ARGS --iqn-head-first $H 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['iqn']['ms_per_step'],4), round(d['iqn']['learn_steps_per_s']))" >> gpurun_out/${T}_ab.txt || exit 2
done; done
cat gpurun_out/${T}_ab.txt
