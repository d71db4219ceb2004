# round 6 head evidence: the full bench line, the AC-IQN step window and kernel stats, the 1-rank RCCL DP rehearsal,
# and a 2-rank gloo launch of the bench on the one GPU (the data_parallel fields at N = 2)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06r
R=$PWD
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], 'iqn', d['iqn']['ms_per_step'], 'rb', d['rainbow']['ms_per_step'], 'dropin', d['dropin_single_env']['env_steps_per_s'])"
(cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/${T}_prof && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv rocpd \
   -- python3 $R/bench.py --steps 50 --warmup 10 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 \
   --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 > $R/gpurun_out/${T}_prof.json 2> $R/gpurun_out/${T}_prof.err) || exit 4
python tools/step_window.py gpurun_out/${T}_prof/run_results.db > gpurun_out/${T}_step_window.txt 2>&1
head -14 gpurun_out/${T}_step_window.txt
cp gpurun_out/${T}_prof/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
BASE="--steps 20 --warmup 5 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 --plateau-envs 0 --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0"
timeout -k 10 300 python -u bench.py --dp-rehearsal $BASE > gpurun_out/${T}_dp_rehearsal.json 2> gpurun_out/${T}_dp.err || { tail -20 gpurun_out/${T}_dp.err; exit 5; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 \
  bench.py --gpus 2 --backend gloo --same-device --steps 10 --warmup 3 --iqn-steps 0 --rainbow-steps 0 --config5-steps 0 \
  --plateau-envs 0 --no-cpu-baseline --no-learn-b64 --fp32-steps 0 --dropin-seconds 0 > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.err || { tail -20 gpurun_out/${T}_gloo2.err; exit 6; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_gloo2.json').read().strip().splitlines()[-1]); print('gloo2', d['ms_per_step'], json.dumps(d.get('data_parallel'))[:600])"
echo done
