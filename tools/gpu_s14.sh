set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s14
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-cpu > $O/bench_prof.json 2> $O/prof.err
