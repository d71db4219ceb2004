#!/bin/bash
# round 3: phase stamps of the actor gradient launch (variant build), with and without the fused optimiser
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r03ag}
OUT=gpurun_out/${T}_stamps.txt
: > $OUT
for m in plain; do
  ASVRL_LIB=variants/libasvrl_agstamps.so timeout -k 10 120 python -u tools/ag_stamps.py $m >> $OUT 2>&1 || exit 2
done
