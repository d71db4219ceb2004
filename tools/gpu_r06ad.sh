# round 6: the pair kernel's launch shape re-swept after the kernarg change (2^18 and 4096 envs, f32 noise)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ad}
for rep in 1 2; do
timeout -k 10 300 python tools/bench_env.py --envs 262144 --noise f32 --iters 20 \
  --launch "1,64,8;1,64,10;1,64,12;1,128,16;1,128,20;1,128,25;1,256,40;1,256,51" 2>/dev/null | python -c "
import json,sys
print(' '.join('%s:%.1fus' % (','.join(map(str,d['launch'])), d['us_per_step']) for d in map(json.loads, sys.stdin)))" >> gpurun_out/${T}_shape.txt || exit 2
timeout -k 10 300 python tools/bench_env.py --envs 4096 --noise f32 --iters 50 \
  --launch "1,256,8;1,256,10;1,256,12;1,128,8;1,64,8;1,64,12;1,128,12" 2>/dev/null | python -c "
import json,sys
print(' '.join('%s:%.1fus' % (','.join(map(str,d['launch'])), d['us_per_step']) for d in map(json.loads, sys.stdin)))" >> gpurun_out/${T}_shape.txt || exit 3
done
cat gpurun_out/${T}_shape.txt
