set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s2/pytest_ring.log 2>&1 &&
timeout -k 10 100 python tools/dbg_compact.py > gpurun_out/s2/dbg.txt 2>&1 &&
timeout -k 10 200 python tools/ab_lookup.py --rounds 7 > gpurun_out/s2/ab.json 2>gpurun_out/s2/ab.err &&
timeout -k 10 200 python tools/ab_lookup.py --rounds 5 --servers 1000 > gpurun_out/s2/ab1000.json 2>>gpurun_out/s2/ab.err
