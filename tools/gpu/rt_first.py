"""Runs bench.py with torch's bundled HIP runtime bound first (import torch before the engine library), to compare
the two HIP runtimes the image holds (torch's ROCm 7.0 copy, the system ROCm 7.2 one bench.py binds by default).
usage: python3 tools/gpu/rt_first.py <bench args>"""
import os
import runpy
import sys

import torch  # noqa: F401  (binds torch/lib/libamdhip64.so before libzbgpu.so's DT_NEEDED runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
