"""Pins the CPU oracle (oracle/msim_oracle.c) before it is trusted as the GPU's checker.

Pins, in order of strength:
  * the reference's own known-answer test, TestSelfishStrategy (test.cpp:213-367), replayed transition by
    transition on the oracle's explicit chains (tests/golden/selfish_strategy_kats.json);
  * outputs of the reference itself recorded in this container: RNG words,
    NextBlockInterval values, PickFinder indices, cumulative thresholds, and all 18 per-miner counters of
    run 0 for two network configurations;
  * the README's published 32768-run averages (statistical, README.md:51-80).
"""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
D = 31_556_952_000


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_rng_kats(oracle):
    b = _load("appendix_b.json")
    for seed, words in b["rng"].items():
        got = oracle.rng_stream(int(seed), 3)
        assert [f"{w:016x}" for w in got] == words


def test_next_block_interval_kat(oracle):
    b = _load("appendix_b.json")
    assert oracle.intervals(1, 6) == b["next_block_interval_rng1_ms"]


def test_pick_finder_kat(oracle):
    b = _load("appendix_b.json")
    assert oracle.picks(b["default9_percs"], 7, 10) == b["pick_finder_default9_rng7"]
    mult = (2**64 - 1) // 100  # simulation.h:18
    cum, thr = 0, []
    for p in b["default9_percs"]:
        cum += p * mult
        thr.append(str(cum))
    assert thr == b["cumulative_thresholds"]


@pytest.mark.parametrize("key,prop", [("run0_prop10s_found_stale", 10_000), ("run0_prop1s_found_stale", 1_000)])
def test_run0_counters_match_reference(oracle, key, prop):
    b = _load("appendix_b.json")
    rc, res, _ = oracle.run(b["default9_percs"], [prop] * 9, [0] * 9, D, *b["run0_seeds"])
    assert rc == 0
    assert res.tolist() == b[key]


def _chain(doc_chain, W):
    out = []
    for blk in doc_chain:
        if blk == "G":
            out.append((0xFFFFFFFF, 0))
        else:
            i, a = blk
            out.append((i, W if a == "W" else a))
    return out


def test_selfish_strategy_kats(oracle):
    """test.cpp:213-367, every case, on the oracle's state machine."""
    doc = _load("selfish_strategy_kats.json")
    W = oracle.SELFISH_ARRIVAL
    sm = doc["selfish_miner"]
    for case in doc["cases"]:
        m = oracle.MinerState(sm["id"], sm["perc"], sm["propagation_ms"], sm["selfish"])
        m.set_chain(_chain(case["chain"], W))
        op = case["op"]
        if op[0] == "found":
            m.found_block(op[1], op[2])
        else:
            m.notify(_chain(op[1], W), op[2])
        assert m.chain() == _chain(case["expect"], W), case["name"]


def test_oracle_vectors_regression(oracle):
    """The committed per-run vectors (tests/golden/oracle_vectors.npz) re-derive from the oracle."""
    z = np.load(os.path.join(GOLD, "oracle_vectors.npz"))
    for name in ("c1_prop10s", "c3_selfish40_prop1s"):
        p, q, s = z[name + "_config"].tolist()
        f, st, _, _ = oracle.run_batch(p, q, s, D, 16, 0, 1000, threads=8)
        assert np.array_equal(f, z[name + "_found"][:16])
        assert np.array_equal(st, z[name + "_stale"][:16])


def test_readme_statistics_10s(oracle):
    """README.md:56,63 (32768 runs, 10 s): miner 0 30.0901% / 1.0092%, miner 7 0.993098% / 1.99286%.
    512 runs here: share within 4 sigma of the binomial MC error, stale rate within 15%."""
    n = 512
    f, st, sh, r = oracle.run_batch([30, 29, 12, 11, 8, 5, 3, 1, 1], [10_000] * 9, [0] * 9, D, n, 0, 77, threads=8)
    share0 = sh[:, 0].mean() * 100
    rate0 = r[:, 0].mean() * 100
    assert abs(share0 - 30.0901) < 4 * 100 * np.sqrt(0.3 * 0.7 / 52_000 / n)
    assert abs(rate0 - 1.0092) / 1.0092 < 0.15
