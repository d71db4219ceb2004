# round 6: where the rollout's replay push waits on the learner -- behind the ACTOR pass (shipped), before it
# (after the critic's Adam; temporary ASVRL_TMP_PUSH_AT=before), or not at all (--push-after-actor 0) --
# alternating, at the driver's shape and at steady state
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ah}
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0"
O=gpurun_out/${T}_push_ab.txt
for shape in "--steps 20 --warmup 5" "--steps 300 --warmup 30"; do
for rep in 1 2 3; do for V in after before none; do
  unset ASVRL_TMP_PUSH_AT; EXTRA=""
  [ $V = before ] && export ASVRL_TMP_PUSH_AT=before
  [ $V = none ] && EXTRA="--push-after-actor 0"
  printf "%s | %s | rep %s: " "$shape" $V $rep >> $O
  timeout -k 10 200 python bench.py $shape $BASE $EXTRA 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> $O || exit 2
done; done; done
cat $O
