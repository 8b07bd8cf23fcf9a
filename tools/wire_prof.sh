set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wprof -o run -- python3 -u bench.py --no-cpu --sim-n 0 --sim5-n 0 --no-merge --steps 3 --warmup 1 > gpurun_out/wprof.json 2> gpurun_out/wprof.err
find gpurun_out/wprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/wprof_stats.csv \;
