set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s27
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
