set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s13
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_lookup.py --rounds 11 --only compact-kpl4/lookupN3,compact-unaligned/lookupN3,compact-kpl2/lookupN3,probe/ablate-hash-only > $O/ab.json 2> $O/ab.err
