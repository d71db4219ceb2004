#!/bin/bash
# GRBM_GUI_ACTIVE per dispatch over the driver-shaped bench run (--steps 20 --warmup 5, main leg only), then the
# fused critic's and the target critic's effective clock over time (tools/clock_probe.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp && rm -rf "$R/gpurun_out/clock"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/clock" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
  --plateau-envs 0 --no-learn-b64 --fp32-steps 0 > "$R/gpurun_out/clock.json" 2> "$R/gpurun_out/clock.err" || exit 1
cd "$R"
f=$(find gpurun_out/clock -name "*counter_collection.csv" | head -1)
python tools/clock_probe.py "$f" --kernel critic_fused_kernel && python tools/clock_probe.py "$f" --kernel "critic_kernel<0"
