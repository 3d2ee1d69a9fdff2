# N=W bench rehearsal on a one-GPU box (all ranks on device 0, gloo-staged halo)
cd $GRAFT_REPO_ROOT
export NBKD_BENCH_SAME_DEVICE=1
W=${W:-4}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus $W --steps 2 --warmup 1 --particles ${N:-5e6} ${BENCH_ARGS} > gpurun_out/n$W.json 2> gpurun_out/n$W.err
rc=$?
tail -5 gpurun_out/n$W.err
cat gpurun_out/n$W.json
exit $rc
