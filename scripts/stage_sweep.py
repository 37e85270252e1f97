import sys, time
sys.path.insert(0, '.')
import torch
torch.cuda.set_device(0)
import miningsimulation_amd as m
rpp = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
sw = m.Sweep(m.c4_grid())
ws = torch.empty(sw.workspace_bytes(rpp), dtype=torch.uint8, device="cuda")
sums = torch.zeros((360, 9, 6), dtype=torch.int64, device="cuda"); st = torch.zeros(2, dtype=torch.int32, device="cuda")
sw.launch(rpp, 0, 1000, sums, ws, st); torch.cuda.synchronize()
t0 = time.perf_counter(); sw.launch(rpp, rpp, 1000, sums, ws, st); torch.cuda.synchronize(); dt = time.perf_counter() - t0
print("sweep 360 x", rpp, "runs:", round(dt, 3), "s ->", round(360 * rpp / dt), "run-years/s; status", st.tolist(), flush=True)
