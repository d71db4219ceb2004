# round 6: Rainbow iterations per captured graph, 2 (default) vs 10 vs 5
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06s
BASE="--no-cpu-baseline --iqn-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 --steps 5 --warmup 2 --rainbow-steps 100"
for rep in 1 2 3; do for U in 2 10 5; do
  printf "unroll %s rep %s: " $U $rep >> gpurun_out/${T}_rb_unroll.txt
  timeout -k 10 200 python bench.py $BASE --rainbow-unroll $U 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['rainbow']['ms_per_step'],4))" >> gpurun_out/${T}_rb_unroll.txt || exit 3
done; done
cat gpurun_out/${T}_rb_unroll.txt
