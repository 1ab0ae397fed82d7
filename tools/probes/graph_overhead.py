"""Where the fixed cost of a short timed region goes (development probe, not
product code): bench.py's default line at --steps K with the timed graph
(a) `default`: as bench.py does it, (b) `prereplay`: the timed graph
replayed once untimed first (diagnosis only — extra warm-up steps, not a
bench.py mode).  A hipGraphUpload of the timed graph at capture (through a
second handle on the HIP runtime) measured no different from (a) and was
dropped.
    python tools/probes/graph_overhead.py MODE K
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def timed_graph_prereplay(step, n, warmup, dist, sync, stream, side=()):
    gw = bench.GraphSteps(step, max(warmup, 1), stream, side=side)
    gm = bench.GraphSteps(step, n, stream, i0=max(warmup, 1), side=side)
    gw.replay()
    gm.replay()
    sync()
    t0 = time.perf_counter()
    gm.replay()
    sync()
    return time.perf_counter() - t0, gm


if __name__ == "__main__":
    mode, k = sys.argv[1], sys.argv[2]
    if mode == "prereplay":
        bench.timed_graph = timed_graph_prereplay
    sys.exit(bench.main(["--no-cpu-baseline", "--no-train", "--steps", k]))
