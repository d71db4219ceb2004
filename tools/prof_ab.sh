#!/bin/bash
# Kernel-trace A/B of tools/bench_critic.py over library variants: bash tools/prof_ab.sh default head bpp4
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=$GRAFT_REPO_ROOT/variants/libasvrl_$L.so; fi
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/pab_$L
  timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pab_$L -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_critic.py --iters 30 > $GRAFT_REPO_ROOT/gpurun_out/pab_$L.log 2>&1
done
