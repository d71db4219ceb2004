set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_mlp_gpu.py tests/test_learner_golden_gpu.py tests/test_agent_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/actor_tests.log 2>&1
rc=$?; tail -2 gpurun_out/actor_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh "default" "sact"
