# env kernel rework: parity tests of every env path, then the plateau sweep over launch shapes
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_env_kernel_gpu.py tests/test_trainer_returns_gpu.py tests/test_dropin_env_gpu.py > gpurun_out/env_try_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_env.py --envs 4096,16384,65536,262144 --noise f32 --launch "auto;1,64,10;1,64,8;1,256,8;1,256,24" > gpurun_out/env_try_base.jsonl 2>&1 && \
timeout -k 10 200 python tools/bench_env.py --envs 262144 --noise f32 --obs-only --launch "1,64,12" > gpurun_out/env_try_obs.jsonl 2>&1 && \
timeout -k 10 200 python tools/bench_env.py --robots 17 --width 110 --envs 4096,65536 --noise f32 --launch "auto;1,256,3;1,256,7;1,256,10" > gpurun_out/env_try_r17.jsonl 2>&1
