#!/bin/bash
# round 3: A/B -- the env step behind the learner's target critic (bench --env-after-target), with and without
# a 16-CU reserve in the fused critic launch (variant build), alternating runs; the chain test for the gate
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03gt}
OUT=gpurun_out/${T}_ab.txt
: > $OUT
for i in 1 2; do
  for cfg in "0 lib/libasvrl.so" "1 lib/libasvrl.so" "1 ../variants/libasvrl_cures16.so" "0 ../variants/libasvrl_cures16.so"; do
    set -- $cfg
    ASVRL_LIB=distributional_rl_decision_and_control_amd/$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
      --plateau-envs 0 --no-cpu-baseline --env-after-target $1 > gpurun_out/${T}_b.json 2> gpurun_out/${T}_b.err || exit 3
    python -c "import json; d=json.loads(open('gpurun_out/${T}_b.json').readline()); print('gate=$1 lib=$2', round(d['ms_per_step'],4), round(d['value']/1e6,3))" >> $OUT
  done
done
cd /tmp && export TMPDIR=/tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/${T}_prof && \
ASVRL_LIB=$GRAFT_REPO_ROOT/variants/libasvrl_cures16.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run --output-format csv rocpd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --env-after-target 1 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.err || exit 4
cd $GRAFT_REPO_ROOT && python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
exit 0
