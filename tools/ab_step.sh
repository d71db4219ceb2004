#!/bin/bash
# A library variant against the default on the bench step (alternating, three reps), after the given tests:
#   TESTS="tests/x.py ..." bash tools/ab_step.sh TAG variant
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; V=$2
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > gpurun_out/${T}_tests.log 2>&1 \
    || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
  tail -1 gpurun_out/${T}_tests.log
fi
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --iqn-steps 200 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2 3; do for L in default $V; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s %s " $rep $L >> gpurun_out/${T}_ab.txt
  timeout -k 10 200 python bench.py $ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']), 'iqn', round(d['iqn']['ms_per_step'],4))" >> gpurun_out/${T}_ab.txt || exit 2
done; done
cat gpurun_out/${T}_ab.txt
