# A/B: observation rows staged in LDS and written once (shipped) vs written in place per phase (variant)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_env_kernel_gpu.py tests/test_trainer_returns_gpu.py tests/test_dropin_env_gpu.py > gpurun_out/env_try_tests.log 2>&1 || exit 1
: > gpurun_out/env_stage_ab.jsonl
for rep in 1 2; do
  for v in base nostage; do
    L=$PWD/distributional_rl_decision_and_control_amd/lib/libasvrl.so; [ $v != base ] && L=$PWD/variants/libasvrl_$v.so
    echo "== $v" >> gpurun_out/env_stage_ab.jsonl
    ASVRL_LIB=$L timeout -k 10 200 python tools/bench_env.py --envs 4096,262144 --noise f32 >> gpurun_out/env_stage_ab.jsonl 2>&1 || exit 1
    ASVRL_LIB=$L timeout -k 10 200 python tools/bench_env.py --robots 17 --width 110 --envs 4096 --noise f32 >> gpurun_out/env_stage_ab.jsonl 2>&1 || exit 1
  done
done
for v in base nostage; do
  L=$PWD/distributional_rl_decision_and_control_amd/lib/libasvrl.so; [ $v != base ] && L=$PWD/variants/libasvrl_$v.so
  ASVRL_LIB=$L PMC_NAME=pmc_stage_$v bash tools/pmc_env.sh > /dev/null 2>&1 || exit 1
done
