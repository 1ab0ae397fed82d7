"""Cost of a stream-ordered hipMemsetAsync of a few bytes in front of a
kernel, inside a HIP graph (development probe): K x (memset 128 B + the
train step) vs K x (train step), eth_hotel_synth shapes.

usage: python tools/probes/memset_cost.py [K]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from multimodaltraj_2_amd import frame_step as fs, train_step as ts  # noqa: E402
from multimodaltraj_2_amd.synthetic import make_batch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda")
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
b = make_batch(256, 32, 128, seed=1)
t = b.to_device(dev)
params = fs.init_params(32, seed=0, device=dev)
st = torch.cuda.Stream(device=dev)
with torch.cuda.stream(st):
    step = ts.TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"], stream=st)
buf = torch.zeros(64, dtype=torch.int32, device=dev)


def run(with_memset):
    if with_memset:
        assert hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, 128, ctypes.c_void_p(st.cuda_stream)) == 0
    step.run()


for name, ms in (("plain", False), ("memset", True), ("plain", False), ("memset", True)):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=st):
        for _ in range(K):
            run(ms)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:7s} {e0.elapsed_time(e1) * 1e3 / K:7.2f} us per train step")
