#!/bin/bash
# IQN stage-ahead A/B: IQN fused / golden tests on the variant, then the IQN training loop (bench_iqn.py) alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ASVRL_LIB=variants/libasvrl_iqnah.so timeout -k 10 300 python -u -m pytest tests/test_iqn_fused_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/iqnah_tests.log 2>&1
rc=$?; tail -2 gpurun_out/iqnah_tests.log; [ $rc -eq 0 ] || exit $rc
for L in cur iqnah cur iqnah cur iqnah; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 120 python tools/bench_iqn.py --iters 300 > gpurun_out/iqnah_$L.json 2>gpurun_out/iqnah_$L.err || exit 1
  echo "$L $(tail -1 gpurun_out/iqnah_$L.json)"
done
