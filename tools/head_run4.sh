#!/bin/bash
# Round-2 head: suite, bench, kernel stats, PMC (head_run2.sh), then the step anatomy (rocpd) and the
# 1-rank RCCL DP rehearsal bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash tools/head_run2.sh > gpurun_out/head_run2.out 2>&1 || { tail -20 gpurun_out/head_run2.out; exit 1; }
tail -2 gpurun_out/head_run2.out
cd $R && bash tools/step_prof.sh && \
cd $R && timeout -k 10 300 python bench.py --dp-rehearsal --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/bench_dp.json 2> gpurun_out/bench_dp.err && tail -1 gpurun_out/bench_dp.json | cut -c1-300
