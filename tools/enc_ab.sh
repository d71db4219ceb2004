#!/bin/bash
# Fused critic: in-kernel encoder gradients (ABI 16) and the next round's input-load position.
# Tests of the fused learner first, then kernel timing / stamps / bench A/B; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_iqn_fused_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
ASVRL_ENC_IN_KERNEL=1 timeout -k 10 400 python -u -m pytest tests/test_learner_golden_gpu.py tests/test_dp_fused_gpu.py tests/test_chain_schedule_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/enc_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/enc_tests2.log; [ $rc -eq 0 ] || exit $rc
for L in default pre1 default pre1; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  timeout -k 10 120 python tools/fused_time.py >> gpurun_out/fused_time.jsonl 2>gpurun_out/fused_time.err || exit 1
done
unset ASVRL_LIB
cat gpurun_out/fused_time.jsonl
for L in stamps stamps1; do
  ASVRL_LIB=variants/libasvrl_$L.so timeout -k 10 200 python tools/fused_stamps.py > gpurun_out/$L.txt 2>&1 || exit 1
  echo "== $L"; grep -v amdgpu gpurun_out/$L.txt
done
for E in 1 0 1 0; do
  ASVRL_ENC_IN_KERNEL=$E timeout -k 10 300 python bench.py --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --iqn-steps 0 > gpurun_out/bench_enc$E.json 2> gpurun_out/bench_enc$E.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_enc$E.json').read().strip().splitlines()[-1]); print('enc=$E', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
done
