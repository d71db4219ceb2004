# round 6: the pair kernel's new automatic launch shape (256 lanes x 10 envs below 16384 envs, 128 lanes x 20 from
# there, R = 5): env parity, the env step and the AC-IQN step against the previous shape rule
# (variants/libasvrl_shapeold.so), then the env PMC passes at both sizes for profiles/r06_env_pmc.json
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ae}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_env_kernel_gpu.py tests/test_dropin_env_gpu.py tests/test_eval_golden_gpu.py tests/test_eval60_golden_gpu.py \
  tests/test_chain_schedule_gpu.py tests/test_batched_eval_gpu.py \
  > gpurun_out/${T}_env_tests.log 2>&1 || { tail -30 gpurun_out/${T}_env_tests.log; exit 2; }
tail -1 gpurun_out/${T}_env_tests.log
O=gpurun_out/${T}_ab.txt
for rep in 1 2 3; do for L in default shapeold; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s rep %s env: " $L $rep >> $O
  timeout -k 10 120 python tools/bench_env.py --envs 4096,262144 --noise f32 --iters 30 2>/dev/null | python -c "
import json,sys
print(' '.join('%d:%.1fus' % (d['envs'], d['us_per_step']) for d in map(json.loads, sys.stdin)))" >> $O || exit 3
  printf "%s rep %s bench: " $L $rep >> $O
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
    --plateau-envs 0 --no-learn-b64 --fp32-steps 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> $O || exit 4
done; done
unset ASVRL_LIB
cat $O
PMC_NAME=${T}_pmc4096 ENV_ARGS="--envs 4096 --noise f32 --iters 3" timeout -k 10 600 bash tools/pmc_env.sh > gpurun_out/${T}_pmc4096.log 2>&1 || exit 5
PMC_NAME=${T}_pmc262k ENV_ARGS="--envs 262144 --noise f32 --iters 3" timeout -k 10 600 bash tools/pmc_env.sh > gpurun_out/${T}_pmc262k.log 2>&1 || exit 6
python tools/pmc_summary.py gpurun_out/${T}_pmc4096 --match env_ --json gpurun_out/${T}_env_pmc_4096.json > gpurun_out/${T}_pmc_summary_4096.txt 2>&1
python tools/pmc_summary.py gpurun_out/${T}_pmc262k --match env_ --json gpurun_out/${T}_env_pmc_262144.json > gpurun_out/${T}_pmc_summary_262144.txt 2>&1
echo done
