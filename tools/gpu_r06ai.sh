# round 6: the next learn step's draw + target actor on the rollout stream behind the push, its actor TRAIN
# forward behind the act (VecTrainer.draw_ahead, ABI 27) -- parity tests, then A/B against the one-launch
# prologue at the head of each learn step, alternating, at the driver's shape and at steady state
# (the --draw-ahead flag and asvrl_learn_prologue_target were removed after this A/B: DESIGN.md section 6)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ai}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_learn_kernels_gpu.py -k "prologue" tests/test_chain_schedule_gpu.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0"
O=gpurun_out/${T}_draw_ahead_ab.txt
for shape in "--steps 20 --warmup 5" "--steps 300 --warmup 30"; do
for rep in 1 2 3; do for V in 1 0; do
  printf "%s | draw_ahead %s | rep %s: " "$shape" $V $rep >> $O
  timeout -k 10 200 python bench.py $shape $BASE --draw-ahead $V 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']), d['config']['draw_ahead'])" >> $O || exit 2
done; done; done
cat $O
