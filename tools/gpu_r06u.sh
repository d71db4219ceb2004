# round 6: env pair kernel register budget (waves per EU 4 = 128 VGPRs, 3 spills; 3 = 134 VGPRs, none)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06u
for rep in 1 2 3; do for L in default wpe3; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s rep %s: " $L $rep >> gpurun_out/${T}_env_wpe.txt
  timeout -k 10 120 python tools/bench_env.py --envs 4096,262144 --noise f32 --iters 30 2>/dev/null | python -c "
import json,sys
print(' '.join('%d:%.1fus' % (d['envs'], d['us_per_step']) for d in map(json.loads, sys.stdin)))" >> gpurun_out/${T}_env_wpe.txt || exit 3
done; done
unset ASVRL_LIB
cat gpurun_out/${T}_env_wpe.txt
