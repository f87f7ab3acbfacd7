cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gnprof_r05
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gnprof_r05 -o gn -- python3 tools/prof_gn.py 10 > gpurun_out/gnprof_r05.log 2>&1
