set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_iqn_gpu.py tests/test_learner_golden_gpu.py tests/test_fused_critic_gpu.py tests/test_iqn_fused_gpu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/act_tests.log 2>&1
rc=$?; tail -3 gpurun_out/act_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline > gpurun_out/bench_act.json 2> gpurun_out/bench_act.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_act.json')); print(d['value'], d['ms_per_step'], d['iqn'])"
