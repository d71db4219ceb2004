# round 6: the partial-sums 16-byte path (a workgroup per 256 outputs of a plain segment, bit-identical to the
# scalar path) -- its tests and the reductions' consumers, then A/B against the scalar path (variant scalarsum)
# (the 16-byte path and its scalarsum variant were removed after this A/B: DESIGN.md section 6)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ak}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_wgrad_gpu.py tests/test_critic_fused_gpu.py tests/test_critic_bf16_oracle_gpu.py \
  tests/test_learner_golden_gpu.py tests/test_iqn_fused_gpu.py tests/test_chain_schedule_gpu.py \
  tests/test_dp_fused_gpu.py tests/test_rainbow_golden_gpu.py > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
REPS=3 bash tools/ab_libs.sh $T default scalarsum
