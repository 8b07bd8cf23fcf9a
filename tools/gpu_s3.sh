set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/pytest_ring.log 2>&1 &&
timeout -k 10 200 python tools/ab_cb.py > gpurun_out/s3/abcb.txt 2>&1
