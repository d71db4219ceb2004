# round 6 final head evidence: the whole -m gpu suite, smoke(), the default bench line, a rocprofv3 kernel trace +
# stats of the AC-IQN loop with one graph-replayed step's window (the trace database removed after, so the
# outputs travel back)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06am}
R=$PWD
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 2; }
tail -1 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 3
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], 'iqn', d['iqn']['ms_per_step'], 'rb', d['rainbow']['ms_per_step'], 'dropin', d['dropin_single_env']['env_steps_per_s'], 'cpu', d['cpu_baseline']['value'])"
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 \
   --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 5
python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
cp gpurun_out/${T}_prof/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
rm -rf gpurun_out/${T}_prof gpurun_out/r06al_prof
head -14 gpurun_out/${T}_step_window.txt
