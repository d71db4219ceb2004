#!/bin/bash
# bench step with the in-launch target critic on / off (alternating): bash tools/ab_tq_bench_only.sh TAG
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2 3; do for V in 1 0; do
  printf "%s target_in_fused=%s " $rep $V >> gpurun_out/${T}_ab.txt
  timeout -k 10 150 python bench.py $ARGS --target-in-fused $V 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> gpurun_out/${T}_ab.txt || exit 2
done; done
cat gpurun_out/${T}_ab.txt
