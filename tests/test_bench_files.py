"""The committed files bench.py reads its roofline constants from exist, parse, and travel to the GPU box: the
driver runs bench.py there from a snapshot of this tree minus .gpurunignore, so an ignore pattern that matches
them leaves every roofline fraction null."""
import fnmatch
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _ignored(rel: str) -> bool:
    """tar --exclude semantics of the patterns gpurun applies: './x' anchors at the top, others match any
    path component suffix."""
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        pats = [p.strip() for p in f if p.strip() and not p.startswith("#")]
    parts = rel.split("/")
    for p in pats:
        if p.startswith("./"):
            q = p[2:].rstrip("/")
            if fnmatch.fnmatch(rel, q) or any(fnmatch.fnmatch("/".join(parts[:i]), q) for i in range(1, len(parts))):
                return True
        elif any(fnmatch.fnmatch("/".join(parts[i:]), p) or fnmatch.fnmatch(parts[i], p) for i in range(len(parts))):
            return True
    return False


def test_bench_constants_present_and_shipped():
    import bench

    for (cfg, n), ent in bench.PMC.items():
        pm = bench.pmc_constants(cfg, n)
        assert pm is not None, (cfg, ent["file"])
        assert pm["valu"] > 0 and pm["fetch_kb"] > 0, pm
        assert not _ignored(pm["src"]), pm["src"]
        for streams in (1, 2):
            rp = bench.rocprof_kernel_ms(cfg, streams)
            assert rp is not None and rp["avg_ms"] > 0, (cfg, streams)
            assert not _ignored(rp["file"]), rp["file"]


def test_ignore_matcher():
    assert _ignored("miningsimulation_amd/csrc/obj/x.o")
    assert _ignored("build/x/y.txt") and _ignored("a/b/var.vo")
    assert not _ignored("miningsimulation_amd/libmsim.so")
