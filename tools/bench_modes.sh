#!/bin/bash
# bench.py in three modes on the GPU box: default (the driver's line), the 1-rank RCCL rehearsal of
# the DP path (all-reduces issued and captured in the graph) and eager (no HIP graph). One summary
# line per mode: value, ms/step, IQN learn-steps/s, Rainbow ms/step, roofline frac, cpu baseline.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_full.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --dp-rehearsal --iqn-steps 20 --rainbow-steps 10 --no-cpu-baseline \
  > gpurun_out/bench_dpr.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --graphs 0 --iqn-steps 20 --rainbow-steps 10 --no-cpu-baseline \
  > gpurun_out/bench_eager.log 2>&1 || exit 1
for f in full dpr eager; do
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
d = json.loads(open(f"gpurun_out/bench_{f}.log").read().strip().splitlines()[-1])
print(f, round(d["value"]), round(d["ms_per_step"], 4), d["iqn"] and round(d["iqn"]["learn_steps_per_s"]),
      d["rainbow"] and round(d["rainbow"]["ms_per_step"], 3), round(d["roofline"]["frac"], 4),
      (d["cpu_baseline"] or {}).get("value"))
PY
done
