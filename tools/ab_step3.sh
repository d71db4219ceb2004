#!/bin/bash
# the default library against two variants on the bench step (AC-IQN and IQN legs), alternating, three reps:
#   bash tools/ab_step3.sh TAG variantA variantB
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; shift
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps 200 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2 3; do for L in default "$@"; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s %s " $rep $L >> gpurun_out/${T}_ab.txt
  timeout -k 10 200 python bench.py $ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']), 'iqn', round(d['iqn']['ms_per_step'],4))" >> gpurun_out/${T}_ab.txt || exit 2
done; done
cat gpurun_out/${T}_ab.txt
