set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s5
timeout -k 10 400 python bench.py > gpurun_out/s5/bench.json 2> gpurun_out/s5/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/s5/prof -o run -- python bench.py --no-cpu > gpurun_out/s5/bench_prof.json 2> gpurun_out/s5/prof.err
