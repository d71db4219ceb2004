#!/bin/bash
# round 3: phase stamps of the fused learn prologue (variant build)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03pro}
OUT=gpurun_out/${T}_stamps.txt
ASVRL_LIB=variants/libasvrl_prostamps.so timeout -k 10 150 python -u tools/prologue_stamps.py > $OUT 2>&1
