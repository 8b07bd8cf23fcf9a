set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s18
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sim_gpu.py tests/test_sim_shard_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/sim_probe.py 100000 1 300 > $O/sim_100000.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/shard8 -o run -- python -u tools/shard_probe.py 100000 8 12 > $O/shard8.log 2>&1
