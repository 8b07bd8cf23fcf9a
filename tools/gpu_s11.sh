set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s11
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sim_gpu.py tests/test_sim_shard_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for n in 10000 20000 100000; do
  timeout -k 10 200 python -u tools/sim_probe.py $n 1 300 > $O/sim_${n}.log 2>&1 || exit 1
done
