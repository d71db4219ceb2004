set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_critic_fused_gpu.py tests/test_iqn_fused_gpu.py tests/test_learner_golden_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fused_tests.log; [ $rc -eq 0 ] || exit $rc
ASVRL_LIB=variants/libasvrl_stamps.so timeout -k 10 200 python tools/fused_stamps.py > gpurun_out/stamps.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/stamps.txt | tail -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_fused.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['iqn']['learn_steps_per_s'])"
