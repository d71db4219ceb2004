# round-6 evidence run: cooperative-capture probe, DP rehearsal, oracle test numbers, kernel trace + step window,
# PMC passes, default bench. Every GPU step under its own limit; stop at the first failure.
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06g
R=$PWD
timeout -k 10 60 ./tools/coop_capture_probe > gpurun_out/${T}_coop_probe.json 2> gpurun_out/${T}_coop_probe.err; echo "coop rc=$?"; cat gpurun_out/${T}_coop_probe.json
timeout -k 10 300 python -u bench.py --dp-rehearsal --steps 20 --warmup 5 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 > gpurun_out/${T}_dp_rehearsal.json 2> gpurun_out/${T}_dp.err || { tail -20 gpurun_out/${T}_dp.err; exit 2; }
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_critic_bf16_oracle_gpu.py tests/test_eval_iqn_golden_gpu.py -s > gpurun_out/${T}_oracle.log 2>&1 || { tail -20 gpurun_out/${T}_oracle.log; exit 3; }
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 \
   --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 4
python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
rm -rf gpurun_out/pmc
BENCH_ARGS="--steps 10 --warmup 5 --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --dropin-seconds 0 --plateau-envs 0" \
  PMC_EXTRA=1 timeout -k 10 900 bash tools/pmc_run.sh || exit 5
python tools/pmc_summary.py gpurun_out/pmc --json gpurun_out/${T}_pmc_summary.json > gpurun_out/${T}_pmc_summary.txt 2>&1
rm -rf gpurun_out/pmc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 6; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['roofline']['traffic'])"
echo done
