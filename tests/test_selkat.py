"""The reference's TestSelfishStrategy (test.cpp:213-367, as data in tests/golden/selfish_strategy_kats.json)
replayed on the PRODUCT's selfish state machines: the entity engine (msim_sel.h: Sel::found / Sel::notify on
the selfish entity) and the settled form (msim_selm.h: SelMacro::transition), through tests/native/selkat.h —
on the host (CPU suite) and as a gfx950 kernel (-m gpu). What each machine cannot represent is named here:

- entity engine: every case. It does not carry the arrival time of a published block below the chain's
  published tip (blocks are (owner, height); only the tip's arrival enters BestChain, main.cpp:68-82), so at
  those heights the test checks only that the reference's block is published at the op's time.
- settled form: a state is a common prefix, a published tie fork and withheld blocks, between finds whose
  consequences have settled. Not representable: b_race_win (a race against a WITHHELD tip; in a settled state
  the tied selfish branch is always published, so FoundBlock's race case simulation.h:66 never applies there).
  d_race_lost, x_lead1_overtaken and x_two_honest_in_a_row deliver two honest blocks in one notify (the second
  find within the first's propagation, which the settled form hands to the engine); they are replayed as the
  composition of two honest transitions and must settle to the same state.
"""
import ctypes
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAXB = 16
W = -2
UNSEEN = -1
NOT_SETTLED = {"b_race_win"}
COMPOSED = {"d_race_lost", "x_lead1_overtaken", "x_two_honest_in_a_row"}


class KatIn(ctypes.Structure):
    _fields_ = [("op", ctypes.c_uint32), ("bcs", ctypes.c_uint32), ("t", ctypes.c_int64), ("prop", ctypes.c_int64),
                ("n", ctypes.c_uint32), ("bn", ctypes.c_uint32), ("own", ctypes.c_uint32 * MAXB),
                ("bown", ctypes.c_uint32 * MAXB), ("arr", ctypes.c_int64 * MAXB), ("barr", ctypes.c_int64 * MAXB)]


class KatOut(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("err", ctypes.c_uint32), ("stale_s", ctypes.c_uint32),
                ("own", ctypes.c_uint32 * (MAXB + 2)), ("arr", ctypes.c_int64 * (MAXB + 2)), ("rep", ctypes.c_uint32),
                ("F", ctypes.c_uint32), ("h", ctypes.c_uint32), ("w", ctypes.c_uint32), ("pend1", ctypes.c_uint32),
                ("sst", ctypes.c_uint32)]


def _doc():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "selfish_strategy_kats.json")))


def _blocks(chain):
    """A KAT chain without genesis as [(owner, arrival)] (arrival W for SELFISH_ARRIVAL)."""
    assert chain[0] == "G"
    return [(b[0], W if b[1] == "W" else b[1]) for b in chain[1:]]


def _inputs(doc):
    sm = doc["selfish_miner"]
    assert sm["id"] == 0 and sm["selfish"]
    ins = (KatIn * len(doc["cases"]))()
    for x, case in zip(ins, doc["cases"]):
        ch = _blocks(case["chain"])
        op = case["op"]
        x.op = 0 if op[0] == "found" else 1
        x.prop = sm["propagation_ms"]
        x.n = len(ch)
        for i, (o, a) in enumerate(ch):
            x.own[i], x.arr[i] = o, a
        if op[0] == "found":
            x.t, x.bcs = op[1], op[2]
        else:
            best = _blocks(op[1])
            x.t, x.bn = op[2], len(best)
            for i, (o, a) in enumerate(best):
                x.bown[i], x.barr[i] = o, a
    return ins


def _settled(exp, public):
    """The settled tuple (F, h, w, honest branch's miner-1 blocks) the chain `exp` reaches once every published
    block is delivered, against the public (honest) chain `public`."""
    w = 0
    while w < len(exp) and exp[len(exp) - 1 - w][1] == W:
        w += 1
    pub = exp[:len(exp) - w]
    if len(pub) > len(public):  # the selfish branch is longer: everybody adopts it
        return len(pub), 0, w, 0
    if len(pub) < len(public):  # it switched to the public chain
        assert pub == public
        return len(public), 0, w, 0
    f = 0
    while f < len(pub) and pub[f] == public[f]:
        f += 1
    return f, len(pub) - f, w, sum(1 for o, _ in public[f:] if o == 1)


def _check(doc, outs):
    for case, o in zip(doc["cases"], outs):
        name = case["name"]
        exp = _blocks(case["expect"])
        op = case["op"]
        t = op[1] if op[0] == "found" else op[2]
        # entity engine: the whole chain
        assert o.err == 0, name
        assert o.n == len(exp), name
        for i, (own, arr) in enumerate(exp):
            assert o.own[i] == own, (name, i)
            if o.arr[i] == UNSEEN:
                assert arr != W and arr <= t, (name, i)  # published below the tip: arrival not carried
            else:
                assert o.arr[i] == arr, (name, i, o.arr[i], arr)
        init = _blocks(case["chain"])
        dropped = sum(1 for i, (own, _) in enumerate(init) if own == 0 and (i >= len(exp) or exp[i][0] != 0))
        assert o.stale_s == dropped, name  # MaybeReorg's stale_blocks (simulation.h:133)
        # settled form
        if name in NOT_SETTLED:
            assert o.rep == 0, name
            continue
        assert o.rep == 1, name
        public = [b for b in init if b[1] != W] if op[0] == "found" else _blocks(op[1])
        F, h, w, p1 = _settled(exp, public)
        assert (o.F, o.h, o.w, o.pend1) == (F, h, w, p1), (name, (o.F, o.h, o.w, o.pend1), (F, h, w, p1))
        assert o.sst == dropped, name


def test_selfish_kats_cover_the_reference_cases():
    doc = _doc()
    names = {c["name"] for c in doc["cases"]}
    assert len(doc["cases"]) == 11 and NOT_SETTLED | COMPOSED <= names


def test_selfish_kats_on_engine_and_settled_form_host(native_tests):
    lib = ctypes.CDLL(native_tests["selkat_host"])
    ib, ob = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.selkat_sizes(ctypes.byref(ib), ctypes.byref(ob)) == MAXB
    assert (ib.value, ob.value) == (ctypes.sizeof(KatIn), ctypes.sizeof(KatOut))
    doc = _doc()
    ins = _inputs(doc)
    outs = (KatOut * len(ins))()
    lib.selkat_run(ins, outs, len(ins))
    _check(doc, outs)


@pytest.mark.gpu
def test_selfish_kats_on_engine_and_settled_form_gpu():
    """The same replay as a gfx950 kernel (tests/native/libselkat_dev.so, built by __graft_entry__.build)."""
    path = os.path.join(ROOT, "tests", "native", "libselkat_dev.so")
    assert os.path.exists(path), "build the device test library first (__graft_entry__.build)"
    lib = ctypes.CDLL(path)
    ib, ob = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.selkat_sizes(ctypes.byref(ib), ctypes.byref(ob)) == MAXB
    assert (ib.value, ob.value) == (ctypes.sizeof(KatIn), ctypes.sizeof(KatOut))
    doc = _doc()
    ins = _inputs(doc)
    outs = (KatOut * len(ins))()
    assert lib.selkat_run_dev(ins, outs, len(ins)) == 0
    _check(doc, outs)
