# round 6: the env kernarg change against the build before it (variants/libasvrl_before.so), each process timing
# the automatic shape four times after a warm-up (the first timings of a process run up to 13 % slower,
# profiles/r06af_env_shape_interleaved.txt)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ag}
for rep in 1 2; do for L in default before; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  for E in 262144 4096; do
    printf "%s rep %s %s: " $L $rep $E >> gpurun_out/${T}_warm_ab.txt
    timeout -k 10 300 python tools/bench_env.py --envs $E --noise f32 --iters 30 --launch "auto;auto;auto;auto;auto" 2>/dev/null | python -c "
import json,sys
print(' '.join('%.1fus' % d['us_per_step'] for d in map(json.loads, sys.stdin)))" >> gpurun_out/${T}_warm_ab.txt || exit 2
  done
done; done
cat gpurun_out/${T}_warm_ab.txt
