# round 6 final bench line at the head
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06x
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], 'iqn', d['iqn']['ms_per_step'], 'rb', d['rainbow']['ms_per_step'], 'dropin', d['dropin_single_env']['env_steps_per_s'], 'b64', d['learn_b64']['learn_steps_per_s'], d['learn_b64']['iqn']['learn_steps_per_s'], d['learn_b64']['rainbow']['learn_steps_per_s'])"
