cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
O="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64"
for rep in 1 2; do
for A in "--steps 20 --warmup 5" "--steps 20 --warmup 25" "--steps 300 --warmup 30"; do
  printf "%s [%s] " $rep "$A" >> gpurun_out/r04j_warm.txt
  timeout -k 10 150 python bench.py $A $O 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> gpurun_out/r04j_warm.txt || exit 1
done; done
cat gpurun_out/r04j_warm.txt
