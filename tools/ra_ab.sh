#!/bin/bash
# Operand read-ahead in the fused critic (ASVRL_READ_AHEAD = D): fused tests on D=2 and D=3, launch timing,
# stamps, bench. Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for L in ra2 ra3; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 300 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_iqn_fused_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${L}_tests.log 2>&1
  rc=$?; echo "$L tests"; tail -1 gpurun_out/${L}_tests.log; [ $rc -eq 0 ] || exit $rc
done
for L in ra0 ra2 ra3 ra0 ra2 ra3; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 120 python tools/fused_time.py >> gpurun_out/ra_time.jsonl 2>gpurun_out/ra_time.err || exit 1
done
cat gpurun_out/ra_time.jsonl
ASVRL_LIB=variants/libasvrl_stampsra2.so timeout -k 10 200 python tools/fused_stamps.py > gpurun_out/stampsra2.txt 2>&1 || exit 1
echo "== stampsra2"; grep -v amdgpu gpurun_out/stampsra2.txt
bash tools/sum_ab.sh ra0 ra2 ra3
