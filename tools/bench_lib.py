"""bench.py against another build of the library (development A/B, not
product code): python tools/bench_lib.py LIB.so [bench.py args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process)
from multimodaltraj_2_amd import _lib  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    _lib._lib = _lib.load(sys.argv[1])
    sys.exit(bench.main(sys.argv[2:]))
