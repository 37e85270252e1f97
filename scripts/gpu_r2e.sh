#!/bin/bash
# A/B of E1 variants on configs[2] (stage timing + status), env-selected.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r2e}; mkdir -p $O

timeout -k 10 300 python -u -m pytest tests/test_gpu_selfish.py -q --timeout 300 --timeout-method thread -m gpu -k "equals_retry" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "" "MSIM_SEL_NA2=1"; do
  env $v timeout -k 10 300 python -u scripts/stage_c3.py 131072 > $O/stage_$v.txt 2>&1 || { cat $O/stage_$v.txt; exit 1; }
  echo "variant [$v]"; grep c3 $O/stage_$v.txt
done
