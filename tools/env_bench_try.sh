# env parity tests, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_env_kernel_gpu.py tests/test_trainer_returns_gpu.py tests/test_dropin_env_gpu.py tests/test_learn_kernels_gpu.py tests/test_per_gpu.py > gpurun_out/env_try_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
