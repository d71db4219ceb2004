#!/bin/bash
# A library variant against the default: the target-critic launch alone (tools/fused_time.py --mode target),
# the ACTOR pass (tools/bench_critic.py) and the bench step, alternating: bash tools/ab_lib.sh TAG variant
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; V=$2
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0"
for L in default $V; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  timeout -k 10 120 python tools/fused_time.py --mode target 2>&1 | grep us_median | tee -a gpurun_out/${T}_ab.txt
  timeout -k 10 120 python tools/bench_critic.py 2>&1 | tail -1 | cut -c1-400 | tee -a gpurun_out/${T}_ab.txt
done
for rep in 1 2 3; do for L in default $V; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s %s " $rep $L >> gpurun_out/${T}_ab.txt
  timeout -k 10 150 python bench.py $ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> gpurun_out/${T}_ab.txt || exit 2
done; done
cat gpurun_out/${T}_ab.txt
