#!/bin/bash
# Round-2 session A: entity-engine parity on MI355X, then a first c3 timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_selfish.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r2a_pytest.log 2>&1 || { tail -40 gpurun_out/r2a_pytest.log; exit 1; }
tail -5 gpurun_out/r2a_pytest.log
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2a_bench_c3.json 2> gpurun_out/r2a_bench_c3.err || { tail -20 gpurun_out/r2a_bench_c3.err; exit 1; }
cat gpurun_out/r2a_bench_c3.json
python -u - <<'PY' > gpurun_out/r2a_timing.txt 2>&1
import sys, time
sys.path.insert(0, '.')
import torch
torch.cuda.set_device(0)
import miningsimulation_amd as m
for name, pts in (("c3", [m.PRESETS["c3"]()]),):
    sim = m.Simulation(pts[0])
    n = 131072
    ws = torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    sums = torch.zeros((9, 6), dtype=torch.int64, device="cuda"); st = torch.zeros(2, dtype=torch.int32, device="cuda")
    sim.launch(n, 0, 1000, sums, ws, st); torch.cuda.synchronize()
    m.timing_enable(True)
    sim.launch(n, n, 1000, sums, ws, st); torch.cuda.synchronize()
    print(name, m.timing_read(), st.tolist(), sim.pipeline_info(n))
sw = m.Sweep(m.c4_grid())
rpp = 2048
ws = torch.empty(sw.workspace_bytes(rpp), dtype=torch.uint8, device="cuda")
sums = torch.zeros((360, 9, 6), dtype=torch.int64, device="cuda"); st = torch.zeros(2, dtype=torch.int32, device="cuda")
sw.launch(rpp, 0, 1000, sums, ws, st); torch.cuda.synchronize()
t0 = time.perf_counter(); sw.launch(rpp, rpp, 1000, sums, ws, st); torch.cuda.synchronize(); dt = time.perf_counter() - t0
print("sweep 360 x", rpp, "runs:", dt, "s ->", 360 * rpp / dt, "run-years/s; status", st.tolist())
PY
cat gpurun_out/r2a_timing.txt
