import sys, time
sys.path.insert(0, '.')
import torch
torch.cuda.set_device(0)
import miningsimulation_amd as m
n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
sim = m.Simulation(m.PRESETS["c3"]())
ws = torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device="cuda")
sums = torch.zeros((9, 6), dtype=torch.int64, device="cuda"); st = torch.zeros(2, dtype=torch.int32, device="cuda")
sim.launch(n, 0, 1000, sums, ws, st); torch.cuda.synchronize()
m.timing_enable(True)
sim.launch(n, n, 1000, sums, ws, st); torch.cuda.synchronize()
print("c3", n, m.timing_read(), "status", st.tolist(), "found/stale", sums[:, :2].sum(1).tolist() if False else sums[:, :2].tolist(), flush=True)
