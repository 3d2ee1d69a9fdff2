set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 600 python3 -u scripts/lib_ab.py --libs prod,collpush0 --rounds 3 -- --n 1e8 > $O/knn.log 2>&1 \
 && timeout -k 10 600 python3 -u scripts/lib_ab.py --libs prod,ballpush0 --rounds 2 -- --n 1e8 --ball 0.01 > $O/ball.log 2>&1 \
 && timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/bench.json 2> $O/bench.err
rc=$?; tail -4 $O/knn.log; tail -3 $O/ball.log; python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['traversal_per_packet'])"; exit $rc
