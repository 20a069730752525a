import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from ntt_amd.ntt import NTTPlan
pl = NTTPlan(1, 24, 4)
t = pl.fill(pl.empty(), "random", seed=2)
torch.cuda.synchronize()
ev = []
for _ in range(40):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); pl.forward(t); b.record(); ev.append((a, b))
torch.cuda.synchronize()
print("per call ms:", " ".join(f"{a.elapsed_time(b):.2f}" for a, b in ev))
