"""Where the fixed cost of a short timed region goes (development probe, not
product code): bench.py's default line at --steps K with the timed graph
(a) `default`: as bench.py does it, (b) `prereplay`: the timed graph
replayed once untimed first (diagnosis only — extra warm-up steps, not a
bench.py mode), (c) `upload`: hipGraphUpload of every captured graph on the
stream its replays run on, through torch's own HIP runtime (soname
libamdhip64.so.7; r5e/r5f loaded a second copy of the runtime by the
unversioned name, which measured nothing), (d) `onstream`: every replay
launched with the capture stream current (bench.py replays on the default
stream).
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


def patch_upload():
    import ctypes
    import torch
    hip = ctypes.CDLL("libamdhip64.so.7")          # torch's runtime (already loaded)
    hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipGraphUpload.restype = ctypes.c_int
    init = bench.GraphSteps.__init__

    def init_upload(self, *a, **k):
        init(self, *a, **k)
        rc = hip.hipGraphUpload(ctypes.c_void_p(self.g.raw_cuda_graph_exec()),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
        torch.cuda.synchronize()
    bench.GraphSteps.__init__ = init_upload


def patch_onstream():
    import torch
    init = bench.GraphSteps.__init__

    def init_keep(self, step, n, stream, *a, **k):
        init(self, step, n, stream, *a, **k)
        self._stream = stream

    def replay(self):
        with torch.cuda.stream(self._stream):
            self.g.replay()
    bench.GraphSteps.__init__ = init_keep
    bench.GraphSteps.replay = replay


if __name__ == "__main__":
    mode, k = sys.argv[1], sys.argv[2]
    if mode == "prereplay":
        bench.timed_graph = timed_graph_prereplay
    if mode == "upload":
        patch_upload()
    if mode == "onstream":
        patch_onstream()
    sys.exit(bench.main(["--no-cpu-baseline", "--no-train", "--steps", k]))
