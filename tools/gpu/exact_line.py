"""bench.run_exact_tree alone (the extras line c1_exact_tree): prints its JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.argv = [sys.argv[0]] + sys.argv[1:]
import bench  # noqa: E402

a = bench.parse()
from zeebe_amd.engine import lib  # noqa: E402

lib()
print(json.dumps(bench.run_exact_tree(a)))
