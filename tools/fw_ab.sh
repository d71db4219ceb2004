set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_iqn_gpu.py tests/test_learner_golden_gpu.py tests/test_fused_critic_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
bash tools/ab_env.sh "default" "fw16" "a16"
for v in default fw16; do
  if [ $v = default ]; then L=""; else L="ASVRL_LIB=variants/libasvrl_$v.so"; fi
  echo -n "$v iqn step: "; env $L timeout -k 10 120 python tools/bench_iqn.py --iters 200 2>&1 | grep -o '"ms_per_iter": [0-9.]*'
done
