"""The product's draw code (msim_draws.h, msim_fastdraw.h; host build) against glibc log1p/llround bit-for-bit: exactly
what the reference calls (xoroshiro128++.h:19, simulation.h:207-209). The GPU build of the same header is
checked in tests/test_gpu_parity.py::test_gpu_log1p_and_intervals."""
import json
import subprocess


def test_log1p_and_interval_bit_exact(native_tests):
    out = subprocess.run([native_tests["draws_check"], "20000000", "8"], capture_output=True, text=True)
    res = json.loads(out.stdout)
    assert res["bad_log1p"] == 0 and res["bad_interval"] == 0, res
    assert res["random"] >= 19_999_992 and res["structured"] > 40_000
    # the draw kernel's fast interval (msim_fastdraw.h): identical results incl. ~1e6 inputs within
    # +-4 ns of a millisecond boundary; its raw error stays far inside the 1 ns acceptance margin
    assert res["bad_fast_interval"] == 0 and res["near_boundary"] > 900_000, res
    assert res["fast_max_err_ns"] < 0.25, res
    # PickFinder by table lookup == the reference's linear scan (random draws + every threshold +-3)
    assert res["bad_picks"] == 0, res
