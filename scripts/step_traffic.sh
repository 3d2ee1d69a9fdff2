# HBM bytes of one whole kNN step (every kernel of nbkd_query_knn at 1e8, k = 32):
# FETCH_SIZE and WRITE_SIZE passes (separate runs) over scripts/knn_time.py with
# 1 and with 3 timed steps; the difference / 2 removes the build and the warmup
# call (scripts/summarize_step.py).  usage (on the box): TAG=r04y bash scripts/step_traffic.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04y}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
st() { # name counter steps
  echo "[step] $1"
  timeout -s KILL 400 rocprofv3 --pmc $2 -d $O/$1 -o run --output-format csv -- python3 scripts/knn_time.py --n 1e8 --k 32 --steps $3 > $O/$1.log 2>&1
}
st f1 FETCH_SIZE 1 && st f3 FETCH_SIZE 3 && st w1 WRITE_SIZE 1 && st w3 WRITE_SIZE 3
