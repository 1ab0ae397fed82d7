import time, sys, torch
sys.path.insert(0, ".")
from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd.synthetic import make_batch
dev = torch.device("cuda")
b = make_batch(256, 32, 128, seed=1)
t = b.to_device(dev)
params = fs.init_params(32, seed=0, device=dev)
s = torch.cuda.Stream()
plans = [fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                     n_frames=t["n_frames"], ped_mask=t["ped_mask"], pred_layout="ped", stream=s) for _ in range(4)]
for p in plans: p.run()
torch.cuda.synchronize()
N = 400
t0 = time.perf_counter()
for i in range(N): plans[i % 4].run()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"CPU enqueue per step {1e6*(t1-t0)/N:.2f} us, wall per step {1e6*(t2-t0)/N:.2f} us")
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
e0.record(s)
for i in range(N): plans[i % 4].run()
e1.record(s); torch.cuda.synchronize()
print(f"event per step {1e3*e0.elapsed_time(e1)/N:.2f} us")
# graph of 20 steps
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    for i in range(20): plans[i % 4].run()
torch.cuda.synchronize()
for _ in range(3): g.replay()
torch.cuda.synchronize()
e0.record(s)
for i in range(N // 20): g.replay()
e1.record(s); torch.cuda.synchronize()
print(f"graph (20 launches): event per step {1e3*e0.elapsed_time(e1)/N:.2f} us")
t0 = time.perf_counter()
for i in range(N // 20): g.replay()
torch.cuda.synchronize()
print(f"graph wall per step {1e6*(time.perf_counter()-t0)/N:.2f} us")
