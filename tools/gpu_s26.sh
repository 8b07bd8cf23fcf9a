set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s26
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
