# round 6: the draw-ahead schedule's chain tests (bit-identity against the joined schedule) and its step window
# (the --draw-ahead flag and asvrl_learn_prologue_target were removed after this A/B: DESIGN.md section 6)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06aj}
R=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_chain_schedule_gpu.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
for V in 1 0; do
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof$V && \
 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_prof$V -o run --output-format rocpd \
   -- python3 $R/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 \
   --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 --draw-ahead $V > $R/gpurun_out/${T}_prof$V.json 2> $R/gpurun_out/${T}_prof$V.err) || exit 4
python tools/step_window.py gpurun_out/${T}_prof$V/run_results.db > gpurun_out/${T}_step_window_draw_ahead$V.txt 2>&1
cat gpurun_out/${T}_step_window_draw_ahead$V.txt
rm -rf gpurun_out/${T}_prof$V
done
