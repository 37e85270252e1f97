"""The product's draw code (msim_draws.h, host build) against glibc log1p/llround bit-for-bit: exactly
what the reference calls (xoroshiro128++.h:19, simulation.h:207-209). The GPU build of the same header is
checked in tests/test_gpu_parity.py::test_gpu_log1p_and_intervals."""
import json
import subprocess


def test_log1p_and_interval_bit_exact(native_tests):
    out = subprocess.run([native_tests["draws_check"], "20000000", "8"], capture_output=True, text=True)
    res = json.loads(out.stdout)
    assert res["bad_log1p"] == 0 and res["bad_interval"] == 0, res
    assert res["random"] >= 19_999_992 and res["structured"] > 40_000
