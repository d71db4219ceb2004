#!/bin/bash
# A/B library variants (variants/libasvrl_<name>.so, "default" = the in-tree build) on the main bench
# step, alternating, plus one kernel-trace per variant: bash tools/ab_bench.sh default v1 v2 ...
set -e
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out"
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0"
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=$ROOT/variants/libasvrl_$L.so; fi
    printf "%s %s " "$rep" "$L"
    timeout -k 10 120 python3 "$ROOT/bench.py" $ARGS | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))"
  done
done
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=$ROOT/variants/libasvrl_$L.so; fi
  rm -rf "$ROOT/gpurun_out/ab_$L"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/ab_$L" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 > "$ROOT/gpurun_out/ab_$L.log" 2>&1
done
