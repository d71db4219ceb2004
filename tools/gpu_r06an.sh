# round 6: HIP runtime knobs not yet measured on the AC-IQN loop (kernel arguments in device memory, the graph
# launcher's batch size, forced graph queues) against the runtime defaults, alternating, two shapes
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06an}
BASE="--no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-learn-b64 --fp32-steps 0 --dropin-seconds 0"
O=gpurun_out/${T}_runtime_knobs_ab.txt
for shape in "--steps 20 --warmup 5" "--steps 300 --warmup 30"; do
for rep in 1 2; do for V in default HIP_FORCE_DEV_KERNARG=1 HIP_FORCE_DEV_KERNARG=0 DEBUG_HIP_GRAPH_BATCH_SIZE=1 DEBUG_HIP_GRAPH_BATCH_SIZE=512 DEBUG_HIP_FORCE_GRAPH_QUEUES=1; do
  printf "%s | %s | rep %s: " "$shape" $V $rep >> $O
  if [ $V = default ]; then E=""; else E="$V"; fi
  timeout -k 10 150 env $E python bench.py $shape $BASE 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['ms_per_step'],4), round(d['value']))" >> $O || { echo "failed" >> $O; }
done; done; done
cat $O
