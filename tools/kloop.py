"""Run the reference-mode step and the train step of one config in a loop
(profiling driver for rocprofv3 counter passes; development tool).

usage: python tools/kloop.py [CONFIG] [REPS]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multimodaltraj_2_amd import frame_step as fs, train_step as ts  # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "eth_hotel_synth"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    c = CONFIGS[cfg]
    S = c["S"] if c["S"] <= 256 else c["S"] // 8
    dev = torch.device("cuda")
    t = make_batch(S, c["Nmax"], c["H"], seed=1).to_device(dev)
    params = fs.init_params(c["Nmax"], seed=0, device=dev)
    plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    tstep = ts.TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    for _ in range(reps):
        plan.run()
    for _ in range(reps):
        tstep.run()
    torch.cuda.synchronize()
    print("done", cfg, reps)


if __name__ == "__main__":
    main()
