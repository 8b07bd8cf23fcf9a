set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s8
timeout -k 10 300 python -u -m pytest tests/test_sim_gpu.py tests/test_sim_shard_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s8/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s8/prof -o run -- python -u tools/sim_probe.py 100000 1 60 > gpurun_out/s8/sim100k.log 2>&1 &&
RP_SIM_CK=lanes timeout -k 10 300 python -u tools/sim_probe.py 100000 1 60 > gpurun_out/s8/sim100k_lanes.log 2>&1
