import fcntl
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _ensure(path: str, builder) -> None:
    if not os.path.exists(path):
        builder()


def _stale(outs) -> bool:
    """True when a header or source the host builds compile is newer than one of their outputs."""
    srcs = []
    for d, exts in ((os.path.join(ROOT, "miningsimulation_amd", "csrc"), (".h",)),
                    (os.path.join(ROOT, "tests", "native"), (".cpp", ".h"))):
        srcs += [os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts)]
    newest = max(os.path.getmtime(f) for f in srcs)
    return min(os.path.getmtime(p) for p in outs) < newest


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle

    _ensure(pyoracle.LIB, pyoracle.build)
    return pyoracle


@pytest.fixture(scope="session")
def native_tests():
    """Test-only host builds: build/libmodel_host.so and build/draws_check."""
    import __graft_entry__ as ge

    lib = os.path.join(ROOT, "build", "libmodel_host.so")
    pipe = os.path.join(ROOT, "build", "libpipeline_host.so")
    chk = os.path.join(ROOT, "build", "draws_check")
    wide = os.path.join(ROOT, "build", "libwide_host.so")
    sel = os.path.join(ROOT, "build", "libsel_host.so")
    gen = os.path.join(ROOT, "build", "libgeneral_host.so")
    kat = os.path.join(ROOT, "build", "libselkat_host.so")
    seg = os.path.join(ROOT, "build", "libselseg_host.so")
    outs = (lib, chk, pipe, wide, sel, gen, kat, seg)
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    # one builder at a time (pytest-xdist workers share build/): the others wait, then find the outputs fresh
    with open(os.path.join(ROOT, "build", ".native_tests.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not all(os.path.exists(p) for p in outs) or _stale(outs):
            ge.build_native_tests()
    return {"model_host": lib, "draws_check": chk, "pipeline_host": pipe, "wide_host": wide, "sel_host": sel,
            "general_host": gen, "selkat_host": kat, "selseg_host": seg}


@pytest.fixture(scope="session")
def msim_lib_path():
    path = os.path.join(ROOT, "miningsimulation_amd", "libmsim.so")
    if not os.path.exists(path):
        jobs = str(max(1, min(16, os.cpu_count() or 8)))
        subprocess.run(["make", "-s", f"-j{jobs}", "-C", os.path.join(ROOT, "miningsimulation_amd", "csrc")], check=True)
    return path
