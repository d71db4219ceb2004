#!/bin/bash
# Fused-critic variant A/B with a bit-identity gate: for each named library (default = the shipped one,
# others variants/libasvrl_<name>.so) dump the reduced gradients (tools/fused_dump.py) and compare them with
# the first library's, then time the launch (tools/fused_time.py), then phase stamps for the stamp builds.
#   bash tools/ab_fused.sh TAG default v1 v2 ... [-- stampsA stampsB ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; shift
LIBS=(); STAMPS=(); mode=libs
for a in "$@"; do
  if [ "$a" = "--" ]; then mode=stamps; continue; fi
  if [ $mode = libs ]; then LIBS+=("$a"); else STAMPS+=("$a"); fi
done
OUT=gpurun_out/${T}_ab.txt
first=""
for L in "${LIBS[@]}"; do
  if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  timeout -k 10 200 python tools/fused_dump.py gpurun_out/${T}_dump_$L.npz > /dev/null 2>gpurun_out/${T}_dump_$L.err || { echo "dump $L failed" >> $OUT; tail -5 gpurun_out/${T}_dump_$L.err; exit 2; }
  if [ -z "$first" ]; then first=$L; else
    echo -n "$L vs $first: " >> $OUT; python tools/fused_dump.py --compare gpurun_out/${T}_dump_$first.npz gpurun_out/${T}_dump_$L.npz | tail -1 >> $OUT
  fi
done
for rep in $(seq 1 ${REPS:-2}); do for L in "${LIBS[@]}"; do
  if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  echo -n "$rep $L " >> $OUT
  timeout -k 10 120 python tools/fused_time.py 2>/dev/null >> $OUT || exit 3
done; done
for L in "${STAMPS[@]}"; do
  export ASVRL_LIB=variants/libasvrl_$L.so
  echo "== stamps $L" >> $OUT
  timeout -k 10 200 python tools/fused_stamps.py 2>&1 | grep -v amdgpu >> $OUT || exit 4
done
cat $OUT
