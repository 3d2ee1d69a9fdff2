# whole-step HBM traffic of the head (scripts/step_traffic.sh), then the
# log-normal kNN phase split.  usage (on the box): TAG=r04y bash scripts/gpu_r04y.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04y}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG bash scripts/step_traffic.sh \
 && echo "[$TAG] lognormal phases" && timeout -k 10 300 python3 scripts/knn_time.py --n 1e8 --lognormal --steps 2 > $O/lognormal.json 2> $O/lognormal.err
rc=$?
tail -1 $O/lognormal.json
exit $rc
