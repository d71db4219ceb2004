# env kernel at 2^18 envs, observation pass alone and the full step: the shipped kernel and diagnostic variants (timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/envdiag.jsonl
for v in ${ENV_VARIANTS:-base}; do
  L=$PWD/distributional_rl_decision_and_control_amd/lib/libasvrl.so; [ $v != base ] && L=$PWD/variants/libasvrl_$v.so
  echo "== $v" >> gpurun_out/envdiag.jsonl
  ASVRL_LIB=$L timeout -k 10 200 python tools/bench_env.py --envs 262144 --noise f32 --obs-only --launch "auto" >> gpurun_out/envdiag.jsonl 2>&1 || exit 1
  ASVRL_LIB=$L timeout -k 10 200 python tools/bench_env.py --envs 262144 --noise f32 --launch "auto" >> gpurun_out/envdiag.jsonl 2>&1 || exit 1
done
