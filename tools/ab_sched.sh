#!/bin/bash
# A/B of a bench.py flag on the main step (alternating, two reps each):
#   bash tools/ab_sched.sh TAG "--target-after-env 0" "--target-after-env 1"
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; shift
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2; do
  for F in "$@"; do
    printf "%s [%s] " "$rep" "$F" >> gpurun_out/${T}_sched.txt
    timeout -k 10 150 python bench.py $ARGS $F 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']), round(d['roofline']['ms_per_launch'],4))" >> gpurun_out/${T}_sched.txt || exit 1
  done
done
cat gpurun_out/${T}_sched.txt
