cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d $R/gpurun_out/pcs_st -o pcs --output-format csv -- python3 scripts/variants.py --n 2e7 --variants 0 > $R/gpurun_out/pcs_st.log 2>&1
echo "stochastic rc=$?"
tail -5 $R/gpurun_out/pcs_st.log
ls -la $R/gpurun_out/pcs_st/* 2>/dev/null | head
