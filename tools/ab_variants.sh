set -e
mkdir -p gpurun_out
for L in default variants/libasvrl_p32.so variants/libasvrl_p41.so variants/libasvrl_p123.so variants/libasvrl_p127.so; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=$L; fi
  echo "== $L"
  timeout -k 10 120 python tools/bench_iqn.py --iters 300
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --iqn-steps 0 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['ms_per_step'], d['learn_step_ms_eager'])"
done
