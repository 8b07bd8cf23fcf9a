set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s15
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ring_gpu.py tests/test_members_gpu.py tests/test_js_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -c "
import bench, json
rpa = bench.load_pkg()
print(json.dumps(bench.merge_bench(rpa, 0)))
" > $O/merge.json 2> $O/merge.err
