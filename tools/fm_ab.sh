#!/bin/bash
# Read-ahead fences letting VALU/SALU through (fm6) vs closed fences (fm0): fused tests on fm6, launch timing, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ASVRL_LIB=variants/libasvrl_fm6.so timeout -k 10 300 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_iqn_fused_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/fm_tests.log 2>&1
rc=$?; tail -1 gpurun_out/fm_tests.log; [ $rc -eq 0 ] || exit $rc
for L in fm0 fm6 fm0 fm6 fm0 fm6; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 120 python tools/fused_time.py >> gpurun_out/fm_time.jsonl 2>gpurun_out/fm_time.err || exit 1
done
cat gpurun_out/fm_time.jsonl
bash tools/sum_ab.sh fm0 fm6
