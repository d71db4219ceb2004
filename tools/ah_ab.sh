#!/bin/bash
# Stage-ahead A/B of the fused critic: the fused-critic tests on the variant, launch timing, stamps, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ASVRL_LIB=variants/libasvrl_ah1.so timeout -k 10 300 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ah_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ah_tests.log; [ $rc -eq 0 ] || exit $rc
for L in default ah1 pre1 default ah1 pre1; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  timeout -k 10 120 python tools/fused_time.py >> gpurun_out/ah_time.jsonl 2>gpurun_out/ah_time.err || exit 1
done
unset ASVRL_LIB; cat gpurun_out/ah_time.jsonl
for L in stamps2 stampsah1; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 200 python tools/fused_stamps.py > gpurun_out/$L.txt 2>&1 || exit 1
  echo "== $L"; grep -v amdgpu gpurun_out/$L.txt
done
bash tools/sum_ab.sh default ah1
