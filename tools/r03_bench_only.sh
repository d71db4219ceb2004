#!/bin/bash
# round 3: the default bench (3 runs) and one graph-replayed step's anatomy
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03b}
OUT=gpurun_out/${T}_runs.txt
: > $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
    --plateau-envs 0 --no-cpu-baseline > gpurun_out/${T}_b.json 2> gpurun_out/${T}_b.err || exit 3
  python -c "import json; d=json.loads(open('gpurun_out/${T}_b.json').readline()); print(round(d['ms_per_step'],4), round(d['value']/1e6,3))" >> $OUT
done
cd /tmp && export TMPDIR=/tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/${T}_prof && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run --output-format csv rocpd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.err || exit 4
cd $GRAFT_REPO_ROOT && python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
exit 0
