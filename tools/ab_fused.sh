#!/bin/bash
# Launch time of the fused critic (tools/fused_time.py) for the shipped library and each named variant
# (variants/libasvrl_<name>.so, tools/build_variant.py): bash tools/ab_fused.sh TAG default v1 v2 ...
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; shift
for L in "$@"; do
  if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  echo -n "$L " >> gpurun_out/${T}_ab.txt
  timeout -k 10 120 python tools/fused_time.py >> gpurun_out/${T}_ab.txt 2>/dev/null || exit 1
done
cat gpurun_out/${T}_ab.txt
