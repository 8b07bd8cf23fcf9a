set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s1/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s1/prof -o run -- python bench.py --no-cpu > gpurun_out/s1/bench_prof.json 2> gpurun_out/s1/prof.err &&
timeout -k 10 200 python tools/sim_probe.py 30000 1 200 > gpurun_out/s1/sim30k.log 2>&1
