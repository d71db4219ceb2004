set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_eval_golden_gpu.py -v -s -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/eval_tests.log 2>&1
rc=$?; tail -30 gpurun_out/eval_tests.log; exit $rc
