#!/bin/bash
# Resident cos-layer fragments on top of stage-ahead: tests on the variant, launch timing, stamps, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ASVRL_LIB=variants/libasvrl_ah1wc.so timeout -k 10 300 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/wc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wc_tests.log; [ $rc -eq 0 ] || exit $rc
for L in ah1 ah1wc ah1 ah1wc ah1 ah1wc; do
  export ASVRL_LIB=variants/libasvrl_$L.so
  timeout -k 10 120 python tools/fused_time.py >> gpurun_out/wc_time.jsonl 2>gpurun_out/wc_time.err || exit 1
done
unset ASVRL_LIB; cat gpurun_out/wc_time.jsonl
ASVRL_LIB=variants/libasvrl_stampsah1wc.so timeout -k 10 200 python tools/fused_stamps.py > gpurun_out/stampsah1wc.txt 2>&1 || exit 1
echo "== stampsah1wc"; grep -v amdgpu gpurun_out/stampsah1wc.txt
bash tools/sum_ab.sh ah1 ah1wc
