cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_env_kernel_gpu.py tests/test_dropin_env_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/env_pairs.log 2>&1 || { tail -30 gpurun_out/env_pairs.log; exit 1; }
tail -2 gpurun_out/env_pairs.log
ASVRL_ENV_PAIRS=0 timeout -k 10 300 python -u -m pytest tests/test_env_kernel_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/env_serial.log 2>&1 || { tail -30 gpurun_out/env_serial.log; exit 1; }
tail -2 gpurun_out/env_serial.log
for P in 1 0; do
  ASVRL_ENV_PAIRS=$P timeout -k 10 120 python -u tools/bench_env.py --envs 4096,65536,262144 --noise f32 --iters 20 || exit 1
  ASVRL_ENV_PAIRS=$P timeout -k 10 120 python -u tools/bench_env.py --envs 4096,65536 --noise f32 --iters 20 --robots 17 --width 110 || exit 1
done
