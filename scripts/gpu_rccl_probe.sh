# the slab gpu tests (incl. RCCL started in a torch process: the image's librccl)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-rcclprobe}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_slab.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/slab_tests.log 2>&1
rc=$?; tail -15 $O/slab_tests.log; exit $rc
