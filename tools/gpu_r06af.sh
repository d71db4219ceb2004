# round 6: env launch shapes interleaved in one process (auto, 128 x 20, 64 x 8, 256 x 10, ...), three passes
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06af}
for L in default shapeold; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
  printf "%s 2^18: " $L >> gpurun_out/${T}_shape.txt
  timeout -k 10 300 python tools/bench_env.py --envs 262144 --noise f32 --iters 20 \
    --launch "auto;1,128,20;1,64,8;auto;1,128,20;1,64,8;auto;1,128,20;1,64,8;1,64,12;1,128,16" 2>/dev/null | python -c "
import json,sys
print(' '.join('%s:%.1fus' % (','.join(map(str,d['launch'])) if d['launch']!='auto' else 'auto', d['us_per_step']) for d in map(json.loads, sys.stdin)))" >> gpurun_out/${T}_shape.txt || exit 2
  printf "%s 4096: " $L >> gpurun_out/${T}_shape.txt
  timeout -k 10 300 python tools/bench_env.py --envs 4096 --noise f32 --iters 50 \
    --launch "auto;1,256,10;1,256,8;auto;1,256,10;1,256,8;auto;1,256,10;1,256,8" 2>/dev/null | python -c "
import json,sys
print(' '.join('%s:%.1fus' % (','.join(map(str,d['launch'])) if d['launch']!='auto' else 'auto', d['us_per_step']) for d in map(json.loads, sys.stdin)))" >> gpurun_out/${T}_shape.txt || exit 3
done
cat gpurun_out/${T}_shape.txt
