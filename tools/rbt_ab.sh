#!/bin/bash
# Rainbow: the default build (weight-fetch ring in the network and training kernels) vs rb4 (network only):
# Rainbow tests on the default, bench Rainbow line alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_rainbow_gpu.py tests/test_learn_kernels_gpu.py tests/test_per_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/rbt_tests.log 2>&1
rc=$?; tail -1 gpurun_out/rbt_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for L in default rb4; do
    if [ "$L" = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=variants/libasvrl_$L.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 4 --iqn-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --rainbow-steps 40 > gpurun_out/rbt_$L.json 2> gpurun_out/rbt_$L.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/rbt_$L.json').read().strip().splitlines()[-1]); print('$L', round(d['rainbow']['ms_per_step'], 4), round(d['rainbow']['env_steps_per_s']))"
  done
done
