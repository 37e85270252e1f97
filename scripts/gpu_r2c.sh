#!/bin/bash
# Round-2 session C: entity engine after the latency fixes: parity subset, stage timing, PMC of E1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py -v --timeout 300 --timeout-method thread -m gpu -k "equals_retry or oracle" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
cat > $O/stage.py <<'PY'
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
print("c3", n, m.timing_read(), "status", st.tolist(), flush=True)
PY
timeout -k 10 300 python -u $O/stage.py 131072 > $O/stage.txt 2>&1 || { cat $O/stage.txt; exit 1; }
cat $O/stage.txt
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $O/p1 -o p1 -- python3 $O/stage.py 32768 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p2 -o p2 -- python3 $O/stage.py 32768 > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
echo done
