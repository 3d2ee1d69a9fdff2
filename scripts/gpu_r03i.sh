# round refresh (gpu_round.sh) + the same-GPU RCCL probe
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03i} bash scripts/gpu_round.sh \
 && echo "[r03i] rccl same-gpu probe" \
 && timeout -k 10 300 python3 -u scripts/rccl_same_gpu.py > gpurun_out/${TAG:-r03i}/rccl_same_gpu.log 2>&1
rc=$?; tail -20 gpurun_out/${TAG:-r03i}/rccl_same_gpu.log; exit $rc
