# N=W bench rehearsals on a one-GPU box (all ranks on device 0, gloo-staged halo):
#   WS="2 4" N=1e8 bash scripts/rehearse_nw.sh   (strong scaling by default, as bench.py)
cd $GRAFT_REPO_ROOT
export NBKD_BENCH_SAME_DEVICE=1
mkdir -p gpurun_out/rehearse
rc=0
for W in ${WS:-4}; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29510 + W)) bench.py --gpus $W --steps ${STEPS:-3} --warmup 1 --particles ${N:-1e8} ${BENCH_ARGS} > gpurun_out/rehearse/n$W.json 2> gpurun_out/rehearse/n$W.err
  rc=$?
  tail -3 gpurun_out/rehearse/n$W.err
  cut -c1-900 gpurun_out/rehearse/n$W.json
  [ $rc -ne 0 ] && break
done
exit $rc
