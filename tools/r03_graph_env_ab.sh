#!/bin/bash
# round 3: the HIP graph executor's queue / batching knobs against the headline bench leg
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03}
O=gpurun_out/${T}_graph_env_ab.txt
: > $O
run() {
  echo "== $*" >> $O
  env "$@" timeout -k 10 120 python -u bench.py --steps 40 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
    --plateau-envs 0 --no-cpu-baseline 2>> gpurun_out/${T}_graph_env_ab.err | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" >> $O || return 1
}
run X=0 && run DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && run DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && \
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && run DEBUG_HIP_GRAPH_BATCH_SIZE=1 && \
run DEBUG_HIP_GRAPH_BATCH_SIZE=64 && run GPU_STREAMOPS_CP_WAIT=1 && run X=0
