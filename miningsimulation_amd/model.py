"""First-order analytical stale-rate model: a cross-check for simulated results.

Restates the closed form of /root/reference/plot_stale_rate/plot.py:18-77 (exp_dist_cdf, p_finds_within,
p_stale_before, p_stale_after, get_stale_rates, get_net_benefits) for ANY network description — the
reference hard-codes its ten pools (plot.py:8-16) — so that the simulator's honest stale rates can be
checked against it, including networks the reference cannot express (BASELINE configs[4], 1 026 miners).

For a miner with hashrate share h and a common propagation delay d (seconds), with network block rate
lambda = 1/600 s:
  p_before(h) = (1 - exp(-lambda (1 - h) d)) * (1 - h)          its block loses a race it was late to
  p_after(h)  = sum_{o != miner} (1 - exp(-lambda h_o d)) * h_o  another miner extends a competing block
  stale(h)    = p_before(h) + p_after(h)
  benefit(h)  = (h (1 - stale(h)) / (1 - sum_o h_o stale(h_o)) - h) / h
It ignores multi-block races and same-miner effects; it agrees with the simulator to first order (SURVEY
§8c: 0.1017 % model vs 0.1018 % simulated at 1 s for the 30 % pool).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

BLOCK_RATE_PER_S = 1.0 / 600.0  # plot.py:5 LAMBDA

# plot.py:8-16: the 2025 pool distribution the reference's plot uses (shares of network hashrate).
REFERENCE_POOLS: Dict[str, float] = {
    "ANTPOOL": 0.3, "FOUNDRY": 0.29, "VIABTC": 0.12, "F2POOL": 0.11, "SPIDER": 0.08, "MARA": 0.05,
    "SECPOOL": 0.03, "SMALL": 0.012, "VERYSMALL": 0.006, "TINY": 0.002,
}


def _p_within(prop_s: float, share: float) -> float:
    """P(a miner with `share` of the hashrate finds a block within prop_s seconds) (plot.py:18-27)."""
    return 1.0 - math.exp(-BLOCK_RATE_PER_S * share * prop_s)


def stale_rates(shares: Sequence[float], prop_s: float) -> List[float]:
    """Model stale rate of every miner (plot.py:29-58), shares summing to ~1, common delay prop_s."""
    after = [_p_within(prop_s, h) * h for h in shares]
    s_after = sum(after)
    out = []
    for h, a in zip(shares, after):
        p_before = _p_within(prop_s, 1.0 - h) * (1.0 - h)
        out.append(p_before + (s_after - a))
    return out


def net_benefits(shares: Sequence[float], prop_s: float) -> List[float]:
    """Relative revenue change of every miner after difficulty adjustment (plot.py:60-77)."""
    st = stale_rates(shares, prop_s)
    total_found = 1.0 - sum(h * r for h, r in zip(shares, st))
    return [((h * (1.0 - r) / total_found) - h) / h if h > 0 else 0.0 for h, r in zip(shares, st)]


def shares_of(miners, total_weight: int = 100) -> List[float]:
    """Hashrate shares of a Miner list (Miner.perc are percentages, or weights summing to total_weight)."""
    return [m.perc / float(total_weight) for m in miners]
