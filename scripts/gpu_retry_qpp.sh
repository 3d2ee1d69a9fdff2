# log-normal kNN: retry packets of 64 vs one query per wave (separate processes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-rqpp}
mkdir -p $O
for Q in 64 1; do
  NBKD_RETRY_QPP=$Q timeout -k 10 300 python -u scripts/variants.py --n ${N:-1e8} --dist lognormal --variants 0 > $O/q$Q.log 2>&1 || { tail -5 $O/q$Q.log; exit 1; }
  echo "QPP=$Q"; tail -1 $O/q$Q.log | cut -c1-420
done
