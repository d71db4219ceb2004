cd $GRAFT_REPO_ROOT
for L in default nocol; do
  if [ $L = default ]; then unset ASVRL_LIB; else export ASVRL_LIB=$GRAFT_REPO_ROOT/build/variants/libasvrl_$L.so; fi
  for P in 1 0; do
    for OO in "" "--obs-only"; do
      ASVRL_ENV_PAIRS=$P timeout -k 10 120 python -u tools/bench_env.py --envs 4096,262144 --noise f32 --iters 20 $OO | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$L', 'pairs=$P', '$OO', d['envs'], round(d['us_per_step'], 1))" || exit 1
    done
  done
done
