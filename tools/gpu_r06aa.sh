# round 6: the fused critic / IQN update kernels reading FusedArgs through the kernarg segment, re-read each round
# (SGPR spills 16 / 67 -> 0). Parity of every fused-critic and IQN path first, then A/B against the previous build
# (variants/libasvrl_cfbefore.so) and the IQN-only form (cfiqnonly): the update launches alone, the IQN loop, the
# AC-IQN bench line.
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06aa}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_critic_fused_gpu.py tests/test_fused_critic_gpu.py tests/test_critic_fused8_gpu.py tests/test_critic_bf16_oracle_gpu.py \
  tests/test_iqn_fused_gpu.py tests/test_fused_iqn_gpu.py tests/test_learner_golden_gpu.py tests/test_chain_schedule_gpu.py \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 2; }
tail -2 gpurun_out/${T}_tests.log
O=gpurun_out/${T}_ab.txt
for rep in 1 2 3; do for L in default cfbefore cfiqnonly; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s rep %s fused: " $L $rep >> $O
  timeout -k 10 180 python tools/ab_fused_variant.py --variants 4 --reps 3 2>/dev/null | tail -1 >> $O || exit 3
  printf "%s rep %s iqn loop: " $L $rep >> $O
  timeout -k 10 180 python tools/bench_iqn.py --iters 200 2>/dev/null | tail -1 >> $O || exit 4
  printf "%s rep %s bench: " $L $rep >> $O
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
    --plateau-envs 0 --no-learn-b64 --fp32-steps 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> $O || exit 5
done; done
unset ASVRL_LIB
cat $O
