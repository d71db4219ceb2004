# round 6: the env PMC at 4096 envs for profiles/r06_env_pmc.json (the 2^18 pass is r06z's), then the full bench line
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=${T:-r06ab}
PMC_NAME=${T}_pmc_env4096 ENV_ARGS="--envs 4096 --noise f32 --iters 3" timeout -k 10 900 bash tools/pmc_env.sh > gpurun_out/${T}_pmc.log 2>&1 || exit 2
python tools/pmc_summary.py gpurun_out/${T}_pmc_env4096 --match env_ --json gpurun_out/${T}_env_pmc_4096.json > gpurun_out/${T}_pmc_summary_4096.txt 2>&1
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
tail -1 gpurun_out/${T}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('roofline_env_plateau',{}).get('frac'), d.get('roofline_env',{}).get('frac'))"
