set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s4
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/s4/pytest.log 2>&1
