#!/bin/bash
# IQN loop with the chained schedule on / off (bench iqn leg, alternating), then one IQN step window
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1
ARGS="--steps 10 --warmup 10 --iqn-steps 300 --no-cpu-baseline --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2; do for C in 0 1; do
  printf "%s chain=%s " $rep $C >> gpurun_out/${T}_ab.txt
  timeout -k 10 200 python bench.py $ARGS --chain $C 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['iqn']['ms_per_step'],4), round(d['iqn']['learn_steps_per_s']))" >> gpurun_out/${T}_ab.txt || exit 2
done; done
cat gpurun_out/${T}_ab.txt
R=$PWD
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
  -- python3 $R/bench.py --steps 10 --warmup 10 --iqn-steps 50 --no-cpu-baseline --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 \
  > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 3
python tools/step_window.py gpurun_out/${T}_prof/run_results.db --anchor "critic_fused_kernel<32, true" --at 0.8 > gpurun_out/${T}_step_window.txt 2>&1; head -30 gpurun_out/${T}_step_window.txt
