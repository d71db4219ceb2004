# round 6: the IQN target in the fused launch at the reference's B = 64 (learn_b64 legs, no rollout beside them)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06k
OUT=gpurun_out/${T}_b64_ab.txt
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --fp32-steps 0 --dropin-seconds 0 --steps 5 --warmup 2"
for rep in 1 2 3; do for V in 0 1; do
  printf "iqn-target-in-fused %s | rep %s: " $V $rep >> $OUT
  timeout -k 10 200 python bench.py $BASE --iqn-target-in-fused $V 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); b=d['learn_b64']; print('ac-iqn', round(b['ms_per_step']*1e3,2), 'iqn', round(b['iqn']['ms_per_step']*1e3,2), 'us')" >> $OUT || exit 3
done; done
cat $OUT
echo done
