"""C3 merge bench alone (for rocprofv3 kernel traces)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

rpa = bench.load_pkg()
print(json.dumps(bench.merge_bench(rpa, 0)))
