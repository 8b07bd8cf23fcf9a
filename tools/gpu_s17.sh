set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sim_gpu.py tests/test_sim_shard_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for m in pc pc3; do
  RP_SIM_CK=$m timeout -k 10 200 python -u tools/sim_probe.py 10000 1 300 > $O/sim_10000_$m.log 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/shard8 -o run -- python -u tools/shard_probe.py 100000 8 12 > $O/shard8.log 2>&1 || exit 1
RP_SIM_CK=pc3 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/shard8_pc3 -o run -- python -u tools/shard_probe.py 100000 8 12 > $O/shard8_pc3.log 2>&1
