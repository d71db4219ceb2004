# round 6: host profile of the drop-in path (dropin_single_env)
set -o pipefail; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; T=r06m
timeout -k 10 300 python -u tools/profile_dropin.py --steps 400 > gpurun_out/${T}_dropin_profile.txt 2>&1 || { tail -20 gpurun_out/${T}_dropin_profile.txt; exit 2; }
head -120 gpurun_out/${T}_dropin_profile.txt
