#!/bin/bash
# A/B library variants (variants/libasvrl_<name>.so) on the IQN and AC-IQN training loops:
#   bash tools/ab_variants.sh default sw16 ...
set -e
mkdir -p gpurun_out
for L in "$@"; do
  if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  echo "== $L"
  timeout -k 10 120 python tools/bench_iqn.py --iters 300
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --iqn-steps 0 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['ms_per_step'], d['learn_step_ms_eager'])"
done
