#!/bin/bash
set -e
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps 200 --rainbow-steps 0"
for rep in 1 2 3; do
  for T in "$ROOT" "$ROOT/variants/prev"; do
    printf "%s %s " "$rep" "$(basename $T)"
    timeout -k 10 150 python3 "$T/bench.py" $ARGS | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['iqn']['ms_per_step'],4))"
  done
done
