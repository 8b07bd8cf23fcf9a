set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s25
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py --steps 2 --warmup 1 --batch-log2 20 --no-merge --sim-n 0 --sim5-n 0 --no-cpu > $O/bench_wire_prof.json 2> $O/bench_wire_prof.err || exit 1
