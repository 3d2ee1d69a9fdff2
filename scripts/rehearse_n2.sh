# N=2 bench rehearsal on a one-GPU box (both ranks on device 0, gloo-staged halo)
cd $GRAFT_REPO_ROOT
export NBKD_BENCH_SAME_DEVICE=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --particles ${N:-2e7} > gpurun_out/n2.json 2> gpurun_out/n2.err
rc=$?
tail -5 gpurun_out/n2.err
cat gpurun_out/n2.json
exit $rc
