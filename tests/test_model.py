"""The first-order analytical model (miningsimulation_amd/model.py, plot.py:18-77 restated) — SURVEY §8 f4.

Pinned by the values the survey recorded from the reference's own plot.py in this container (SURVEY §8c:
0.1017 % at 1 s and 1.0125 % at 10 s for the 30 % pool), and cross-checked against the oracle's simulated
stale rates (first-order agreement only: the model ignores multi-block races)."""
import numpy as np
import pytest

from miningsimulation_amd import model


def test_reference_pool_values():
    sh = list(model.REFERENCE_POOLS.values())
    assert round(model.stale_rates(sh, 1.0)[0] * 100, 4) == 0.1017
    assert round(model.stale_rates(sh, 10.0)[0] * 100, 4) == 1.0125


def test_net_benefits_conserve_share():
    """After difficulty adjustment the accepted shares sum to 1 (plot.py:64-77)."""
    for shares in (list(model.REFERENCE_POOLS.values()), [30720 / 102400, 29696 / 102400] + [41 / 102400] * 1024):
        for d in (0.1, 1.0, 30.0):
            b = model.net_benefits(shares, d)
            assert abs(sum(h * (1 + x) for h, x in zip(shares, b)) - 1.0) < 1e-12
            assert b[0] > 0 > b[-1]  # big pools gain, small miners lose (README.md:72-80)


@pytest.mark.parametrize("prop_ms", [1000, 10_000])
def test_model_vs_oracle_simulation(oracle, prop_ms):
    """Simulated stale rates of the 9-miner network (oracle, 256 runs x 1 year) vs the model."""
    p = [30, 29, 12, 11, 8, 5, 3, 1, 1]
    f, s, sh, r = oracle.run_batch(p, [prop_ms] * 9, [0] * 9, 31_556_952_000, 256, 0, 1000, threads=8)
    sim = r.mean(axis=0)
    mod = np.array(model.stale_rates([x / 100 for x in p], prop_ms / 1000))
    # the three largest pools: enough stale blocks for a 10 % statistical band
    assert np.all(np.abs(sim[:3] / mod[:3] - 1) < 0.10), (sim[:3], mod[:3])
