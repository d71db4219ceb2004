#!/bin/bash
# round 3: fused-critic phase stamps (variant library) + one graph-replayed AC-IQN step's kernels (rocprofv3)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r03}
ASVRL_LIB=variants/libasvrl_stamps.so timeout -k 10 200 python tools/fused_stamps.py > gpurun_out/${T}_stamps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/${T}_prof && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run --output-format csv rocpd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.err || exit 2
cd $GRAFT_REPO_ROOT && DB=$(ls gpurun_out/${T}_prof/*/*.db gpurun_out/${T}_prof/*.db 2>/dev/null | head -1); echo "db=$DB"
python tools/prof_step.py $DB --anchor env_pairs_kernel --index -12 > gpurun_out/${T}_step_anatomy.txt 2>&1
python tools/prof_step.py $DB --anchor env_pairs_kernel --index -22 >> gpurun_out/${T}_step_anatomy.txt 2>&1
exit 0
