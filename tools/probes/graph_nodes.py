"""Diagnose bench.GraphSteps(per_step=True) on a multi-stream capture: every
node's type in hipGraphGetNodes order, each step's nodes,
and which steps' outputs a replay with some nodes disabled writes."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from tests.test_bench_graph_gpu import _plans  # noqa: E402

gpu = torch.device("cuda:0")
for ns in (1, 2):
    streams = [torch.cuda.Stream(device=gpu) for _ in range(ns)]
    plans = _plans(gpu, streams)
    K = len(plans)
    g = bench.GraphSteps(lambda i: plans[i % K].run(), K, streams[0], side=streams[1:], per_step=True)
    graph = ctypes.c_void_p(g.g.raw_cuda_graph())
    cnt = ctypes.c_size_t(0)
    bench.hip().hipGraphGetNodes(graph, None, ctypes.byref(cnt))
    nodes = (ctypes.c_void_p * cnt.value)()
    bench.hip().hipGraphGetNodes(graph, nodes, ctypes.byref(cnt))
    types = []
    for i in range(cnt.value):
        t = ctypes.c_int(-1)
        bench.hip().hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t))
        types.append(t.value)
    print("streams", ns, "types", types)
    print("  step_nodes idx", [[list(nodes).index(n) for n in sn] for sn in g.step_nodes])
    for only in ([1, 2], [0], []):
        for p in plans:
            p.out.h.fill_(float("nan"))
        torch.cuda.synchronize()
        g.replay_only(only)
        print("  only", only, "written", [not bool(torch.isnan(p.out.h).all()) for p in plans])
