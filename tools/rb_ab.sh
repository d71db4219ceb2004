#!/bin/bash
# Kernel-trace A/B of the Rainbow section: bash tools/rb_ab.sh (ASVRL_RAINBOW_SPLITK 0 and 1)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for V in ${VARIANTS:-0 1}; do
  export ASVRL_RAINBOW_GROUP_ROWS=${V#g}
  rm -rf $R/gpurun_out/rb_$V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rb_$V -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --iqn-steps 0 --no-cpu-baseline > $R/gpurun_out/rb_$V.json 2> $R/gpurun_out/rb_$V.err || exit $?
done
