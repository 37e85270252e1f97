"""Writes selfish_strategy_kats.json: the known-answer transitions of the reference's only asserting
test, TestSelfishStrategy (/root/reference/test.cpp:213-367), as data (initial chain, operation,
expected chain). Blocks are [miner_id, arrival_ms]; "G" is Genesis (simulation.h:31-33) and "W" the
SELFISH_ARRIVAL sentinel (simulation.h:20). The selfish miner is Miner{0, 35, 100ms, true} (test.cpp:215-217).
"""
import json
import os

S = 600_000          # 600s in ms (test.cpp uses 600s * k)
P = 100              # SM_PROP_TIME (test.cpp:216)
G = "G"
W = "W"
SM, OT = 0, 1


def b(i, a):
    return [i, a]


cases = [
    # Case (a), test.cpp:219-228
    dict(name="a_found_no_fork", src="test.cpp:221-228", chain=[G, b(OT, S), b(SM, 2 * S)],
         op=["found", 3 * S, 3], expect=[G, b(OT, S), b(SM, 2 * S), b(SM, W)]),
    # Case (a) continued, test.cpp:230-235
    dict(name="a_found_lead1", src="test.cpp:230-235", chain=[G, b(OT, S), b(SM, 2 * S), b(SM, W)],
         op=["found", 4 * S, 3], expect=[G, b(OT, S), b(SM, 2 * S), b(SM, W), b(SM, W)]),
    # Case (b), test.cpp:237-247 (the is_race branch, simulation.h:66-69)
    dict(name="b_race_win", src="test.cpp:239-247", chain=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, W)],
         op=["found", 6 * S, 5],
         expect=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, 6 * S + P), b(SM, 6 * S + P)]),
    # Case (d), test.cpp:252-260
    dict(name="d_race_lost", src="test.cpp:254-260", chain=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, W)],
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(OT, 4 * S), b(OT, 5 * S)], 5 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(OT, 4 * S), b(OT, 5 * S)]),
    # Case (e), test.cpp:262-271
    dict(name="e_no_private_branch", src="test.cpp:264-271",
         chain=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, 4 * S)],
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, 4 * S), b(OT, 5 * S)], 5 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, 4 * S), b(OT, 5 * S)]),
    # Case (f), test.cpp:273-283
    dict(name="f_lead1_reveal", src="test.cpp:276-283", chain=[G, b(OT, S), b(SM, 2 * S), b(SM, W)],
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S)], 3 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(SM, 3 * S + P)]),
    # Case (g), test.cpp:285-296
    dict(name="g_lead2_reveal_all", src="test.cpp:289-296", chain=[G, b(OT, S), b(SM, 2 * S), b(SM, W), b(SM, W)],
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S)], 3 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(SM, 3 * S + P), b(SM, 3 * S + P)]),
    # Case (h), test.cpp:298-314
    dict(name="h_lead3_reveal_one", src="test.cpp:301-314",
         chain=[G, b(OT, S), b(SM, 2 * S), b(SM, W), b(SM, W), b(SM, W)],
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S)], 3 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(SM, 3 * S + P), b(SM, W), b(SM, W)]),
    # Case (h), second form, test.cpp:316-330
    dict(name="h_lead5_reveal_one", src="test.cpp:317-330",
         chain=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S)] + [b(SM, W)] * 5,
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(OT, 4 * S)], 4 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, 4 * S + P)] + [b(SM, W)] * 4),
    # Paper-absent: two honest blocks in a row, test.cpp:332-350
    dict(name="x_two_honest_in_a_row", src="test.cpp:334-350",
         chain=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S)] + [b(SM, W)] * 5,
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(OT, 4 * S), b(OT, 5 * S)], 5 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, 5 * S + P), b(SM, 5 * S + P)] + [b(SM, W)] * 3),
    # Paper-absent: lead 1, two honest blocks in a row, test.cpp:352-364
    dict(name="x_lead1_overtaken", src="test.cpp:354-364",
         chain=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(SM, W)],
         op=["notify", [G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(OT, 4 * S), b(OT, 5 * S)], 5 * S],
         expect=[G, b(OT, S), b(SM, 2 * S), b(OT, 3 * S), b(OT, 4 * S), b(OT, 5 * S)]),
]

doc = {"source": "/root/reference/test.cpp:213-367 TestSelfishStrategy", "selfish_miner": {"id": SM, "perc": 35,
       "propagation_ms": P, "selfish": True}, "cases": cases}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "selfish_strategy_kats.json"), "w") as f:
    json.dump(doc, f, indent=1)
