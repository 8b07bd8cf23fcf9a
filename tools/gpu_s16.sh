set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sim_gpu.py tests/test_sim_shard_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for n in 10000 100000; do
  timeout -k 10 200 python -u tools/sim_probe.py $n 1 300 > $O/sim_${n}.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof100k -o run -- python -u tools/sim_probe.py 100000 1 300 > $O/prof100k.log 2>&1
