# Every rank's slab of the N-GPU bench alone on this one GPU (knn_time.py,
# phase timers on): N = 8, 4, 2 strong, C4 weak (1.25e8 per rank) rank 3, and
# N = 1.  One JSON line per run into gpurun_out/$TAG/slab_ranks.log.
#   usage (on the box): TAG=r06n bash scripts/slab_ranks.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-run}
O=gpurun_out/$TAG
mkdir -p $O
L=$O/slab_ranks.log
: > $L
run() { # knn_time args...
  echo "### $*" >> $O/slab_ranks.err
  timeout -k 10 300 python3 -u scripts/knn_time.py --steps 3 "$@" >> $L 2>> $O/slab_ranks.err
}
for w in 8 4 2; do
  r=0
  while [ $r -lt $w ]; do
    run --n 1e8 --slab-world $w --slab-rank $r || exit $?
    r=$((r + 1))
  done
done
run --n 1.25e8 --slab-world 8 --slab-rank 3 --scaling weak || exit $?
run --n 1e8 || exit $?
