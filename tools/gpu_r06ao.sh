# round 6: the HIP graph launcher's batch size (DEBUG_HIP_GRAPH_BATCH_SIZE) at the driver's shape -- confirming
# r06an's first look (512 ahead of the default by ~2 % over 2 reps), 4 alternating reps per value
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ao}
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --dropin-seconds 0"
O=gpurun_out/${T}_graph_batch_ab.txt
for rep in 1 2 3 4; do for V in default 512 4096 128; do
  printf "driver shape | batch %s | rep %s: " $V $rep >> $O
  if [ $V = default ]; then E=""; else E="DEBUG_HIP_GRAPH_BATCH_SIZE=$V"; fi
  timeout -k 10 150 env $E python bench.py --steps 20 --warmup 5 $BASE 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> $O || { echo "failed" >> $O; }
done; done
cat $O
