set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s7
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s7/pytest.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/s7/bench.json 2> gpurun_out/s7/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/s7/prof -o run -- python bench.py --no-cpu > gpurun_out/s7/bench_prof.json 2> gpurun_out/s7/prof.err
