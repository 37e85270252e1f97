#!/bin/bash
# c2/c3 bench lines with 1 and 2 streams, and the PMC passes of c2's draw kernel (traffic + instruction
# mix) behind the bench line's traffic and issue-fraction constants (profiles/r02/pmc_q.md).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc}; mkdir -p $O
for c in c2 c3; do for st in 1 2; do
  timeout -k 10 300 python -u bench.py --config $c --streams $st --no-cpu-baseline > $O/bench_${c}_s$st.json 2> $O/bench_${c}_s$st.err || { tail -30 $O/bench_${c}_s$st.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${c}_s$st.json'));print('$c streams=$st',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['k1_ms'])"
done; done
P="python3 bench.py --config c2 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o f -- $P > $O/pmc_f.log 2>&1 || { tail -5 $O/pmc_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o w -- $P > $O/pmc_w.log 2>&1 || { tail -5 $O/pmc_w.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_s -o s -- $P > $O/pmc_s.log 2>&1 || { tail -5 $O/pmc_s.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_m -o m -- $P > $O/pmc_m.log 2>&1 || { tail -5 $O/pmc_m.log; echo "mix pass failed (continuing)"; }
find $O -name "*counter_collection.csv" | head
