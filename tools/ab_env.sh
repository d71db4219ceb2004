#!/bin/bash
# A/B of library variants and environment settings on the main bench step, alternating:
#   bash tools/ab_env.sh "default" "c22" "default ASVRL_ACTOR_FWD_SIDE=0" ...
# each argument: a variant name (variants/libasvrl_<name>.so, "default" = in-tree) then VAR=VALUE pairs.
set -e
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps ${IQN_STEPS:-0} --rainbow-steps 0 --config5-steps 0 --plateau-envs 0"
SPECS=("$@")
for rep in 1 2; do
  for spec in "${SPECS[@]}"; do
    set -- $spec
    L=$1; shift
    if [ "$L" = default ]; then LIBV=""; else LIBV="ASVRL_LIB=$ROOT/variants/libasvrl_$L.so"; fi
    printf "%s [%s] " "$rep" "$spec"
    env $LIBV "$@" timeout -k 10 120 python3 "$ROOT/bench.py" $ARGS | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']), (d.get('iqn') or {}).get('ms_per_step'))"
  done
done
