# round 6: env pair kernels reading their arguments per phase / per loop iteration from the kernarg segment
# parity first (env kernel, drop-in env, eval goldens, chain schedule), then an alternating A/B against the
# previous build (variants/libasvrl_before.so), then the env PMC passes of the new build
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06z}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_env_kernel_gpu.py tests/test_dropin_env_gpu.py tests/test_eval_golden_gpu.py tests/test_eval60_golden_gpu.py \
  tests/test_eval_iqn_golden_gpu.py tests/test_chain_schedule_gpu.py tests/test_batched_eval_gpu.py \
  > gpurun_out/${T}_env_tests.log 2>&1 || { tail -30 gpurun_out/${T}_env_tests.log; exit 2; }
tail -3 gpurun_out/${T}_env_tests.log
for rep in 1 2 3; do for L in default before; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s rep %s: " $L $rep >> gpurun_out/${T}_env_ab.txt
  timeout -k 10 120 python tools/bench_env.py --envs 4096,262144 --noise f32 --iters 30 2>/dev/null | python -c "
import json,sys
print(' '.join('%d:%.1fus' % (d['envs'], d['us_per_step']) for d in map(json.loads, sys.stdin)))" >> gpurun_out/${T}_env_ab.txt || exit 3
done; done
unset ASVRL_LIB
cat gpurun_out/${T}_env_ab.txt
PMC_NAME=${T}_pmc_env timeout -k 10 900 bash tools/pmc_env.sh > gpurun_out/${T}_pmc.log 2>&1 || exit 4
python tools/pmc_summary.py gpurun_out/${T}_pmc_env --match env_ --json gpurun_out/${T}_env_pmc.json > gpurun_out/${T}_pmc_summary.txt 2>&1
head -40 gpurun_out/${T}_pmc_summary.txt
