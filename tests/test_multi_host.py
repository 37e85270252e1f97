"""The communicator cache of msim_run_multi (csrc/msim_commcache.h, used by csrc/msim_multi.hip) on the host:
threads sharing one device list, some calls failing their collective and retiring the set. A retired set is
destroyed under its lock, so no caller ever runs a collective on a destroyed communicator. The
reference's counterpart is the std::async fan-out of main.cpp:205-209, whose batches share nothing."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "commcache_host.cpp")


def _run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    ok, calls, inits, destroys = r.stdout.split()
    assert ok == "OK"
    assert int(inits) == int(destroys)  # every stand-in communicator destroyed exactly once, after its last use
    return int(calls)


def test_commcache_retire_under_lock():
    exe = os.path.join(ROOT, "build", "commcache_host")
    if not os.path.exists(exe):
        pytest.skip("build() not run")
    assert _run(exe, 8, 4000) == 32000


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_commcache_thread_sanitizer():
    """The same driver under ThreadSanitizer (host code only): no data race on the entries."""
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "cc_tsan")
        b = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=thread", SRC, "-o", exe],
                           capture_output=True, text=True)
        if b.returncode != 0:
            pytest.skip("ThreadSanitizer unavailable: " + b.stderr[-300:])
        assert _run(exe, 4, 1500) == 6000
