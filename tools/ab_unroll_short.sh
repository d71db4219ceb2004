#!/bin/bash
# iterations per captured graph for the driver's short timed region (--steps 20 --warmup 5), alternating
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2 3; do for U in 10 5 4 2; do
  printf "%s unroll=%s " $rep $U >> gpurun_out/${T}_ab.txt
  timeout -k 10 200 python bench.py $ARGS --unroll $U 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']), d['config']['unroll'])" >> gpurun_out/${T}_ab.txt || exit 2
done; done
cat gpurun_out/${T}_ab.txt
