cd $GRAFT_REPO_ROOT
run() {  # label, env..., args
  local lab="$1"; shift
  env "$@" timeout -k 10 120 python -u tools/bench_env.py --noise f32 --iters 20 $EXTRA | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$lab', d['robots'], d['envs'], round(d['us_per_step'], 1), round(d['env_steps_per_s'] / 1e6, 1))" || exit 1
}
export EXTRA="--envs 4096,65536 --robots 17 --width 110"
run b256e3 ASVRL_ENV_BLK=256 ASVRL_ENV_EPB=3
run b256e1 ASVRL_ENV_BLK=256 ASVRL_ENV_EPB=1
run b128e1 ASVRL_ENV_BLK=128 ASVRL_ENV_EPB=1
run b128e2 ASVRL_ENV_BLK=128 ASVRL_ENV_EPB=2
export EXTRA="--envs 4096,65536,262144"
run b256e12 ASVRL_ENV_BLK=256 ASVRL_ENV_EPB=12
run b128e12 ASVRL_ENV_BLK=128 ASVRL_ENV_EPB=12
run b256e8 ASVRL_ENV_BLK=256 ASVRL_ENV_EPB=8
run b128e8 ASVRL_ENV_BLK=128 ASVRL_ENV_EPB=8
