#!/bin/bash
# Library variants (variants/libasvrl_<name>.so, tools/build_variant.py; "default" = the shipped library)
# on the main AC-IQN leg, alternating, REPS reps (default 2), at the driver's shape and at steady state; then a
# rocprofv3 kernel trace of the shipped library with one graph-replayed step's window (tools/step_window.py).
#   bash tools/ab_libs.sh TAG default VARIANT ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
T=$1; shift
OUT=gpurun_out/${T}_ab.txt
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0"
for shape in "--steps 20 --warmup 5" "--steps 300 --warmup 30"; do
  for rep in $(seq 1 ${REPS:-2}); do for L in "$@"; do
    if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
    printf "%s | %s | rep %s: " "$shape" "$L" "$rep" >> $OUT
    timeout -k 10 200 python bench.py $shape $BASE 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> $OUT || exit 2
  done; done
done
unset ASVRL_LIB
R=$PWD
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py --steps 50 --warmup 10 $BASE > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 4
python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
cat $OUT; head -20 gpurun_out/${T}_step_window.txt
