#!/bin/bash
# Round-2 head: fused-kernel timing vs the previous loss shuffles (pre1 variant), GPU test suite,
# default bench, rocprofv3 kernel stats of the bench, PMC traffic passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && for L in default pre1 default pre1; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  timeout -k 10 120 python tools/fused_time.py >> gpurun_out/fused_time3.jsonl 2>gpurun_out/fused_time3.err || exit 1
done
unset ASVRL_LIB
cat gpurun_out/fused_time3.jsonl
bash tools/head_run2.sh
