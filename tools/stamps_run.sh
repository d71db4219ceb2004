set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ASVRL_LIB=variants/libasvrl_stamps.so timeout -k 10 200 python tools/fused_stamps.py > gpurun_out/stamps.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/stamps.txt | tail -10; exit $rc
