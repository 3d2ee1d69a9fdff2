# kNN A/B runs (one process per setting): TAG=x ENVS="A=1 A=2" EXTRA="--lognormal" bash scripts/gpu_knn_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-knnab}
mkdir -p $O
for L in ${LEAVES:-64}; do
  for E in ${ENVS:-NONE=0}; do
    env $E timeout -k 10 400 python -u scripts/knn_ab.py --n ${N:-1e8} --leaf $L $EXTRA >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  done
done
cat $O/ab.log
