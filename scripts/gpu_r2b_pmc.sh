#!/bin/bash
# Round-2 session B: rocprofv3 kernel stats + PMC passes of the entity engine on configs[2] (32768 runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
cat > gpurun_out/r2b/c3.py <<'PY'
import sys
sys.path.insert(0, '.')
import torch
torch.cuda.set_device(0)
import miningsimulation_amd as m
sim = m.Simulation(m.PRESETS["c3"]())
n = 32768
ws = torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device="cuda")
sums = torch.zeros((9, 6), dtype=torch.int64, device="cuda"); st = torch.zeros(2, dtype=torch.int32, device="cuda")
sim.launch(n, 0, 1000, sums, ws, st); torch.cuda.synchronize()
print("status", st.tolist())
PY
timeout -k 10 120 rocprofv3 -L > gpurun_out/r2b/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b/kt -o kt -- python3 gpurun_out/r2b/c3.py > gpurun_out/r2b/kt.log 2>&1 || { tail -20 gpurun_out/r2b/kt.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH -d gpurun_out/r2b/p1 -o p1 -- python3 gpurun_out/r2b/c3.py > gpurun_out/r2b/p1.log 2>&1 || { tail -20 gpurun_out/r2b/p1.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r2b/p2 -o p2 -- python3 gpurun_out/r2b/c3.py > gpurun_out/r2b/p2.log 2>&1 || { tail -20 gpurun_out/r2b/p2.log; exit 1; }
find gpurun_out/r2b -name "*.csv" | head -20
