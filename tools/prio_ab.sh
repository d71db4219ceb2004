set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
IQN_STEPS=20 bash tools/ab_env.sh "default ASVRL_STREAM_PRIO=1" "default ASVRL_STREAM_PRIO=0"
