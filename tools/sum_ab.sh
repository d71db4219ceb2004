#!/bin/bash
# Partial-sum reduction A/B (loads in flight per wave / waves per output block): AC-IQN bench step
# over library variants, alternating, twice each. bash tools/sum_ab.sh default sacc16 sacc32 swav16
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
    timeout -k 10 300 python bench.py --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --iqn-steps 20 > gpurun_out/sum_$L.json 2> gpurun_out/sum_$L.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/sum_$L.json').read().strip().splitlines()[-1]); print('$L', round(d['value']), round(d['ms_per_step'], 4), d['iqn']['learn_steps_per_s'])"
  done
done
