"""INTEGRATION.md's C++ snippets compile verbatim against include/msim.h (and RCCL / HIP for §3).

Each ```cpp block is pasted unchanged into a harness translation unit that supplies only the context
the doc assumes around it (a reference-shaped Miner list from SetupMiners(), SIM_DURATION, SIM_RUNS
(main.cpp:7-10, 44-65), an RCCL communicator and a HIP stream), then checked with -fsyntax-only.
A signature drift between the doc and the header fails here."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = r"""
#include <chrono>
#include <cstdint>
#include <iostream>
#include <vector>
#include "msim.h"
// Context of the reference's main.cpp the snippets are written against (shape only).
struct RefMiner {
    unsigned id;
    uint64_t perc;
    std::chrono::milliseconds propagation;
    bool is_selfish;
};
static std::vector<RefMiner> SetupMiners() { return {{0, 100, std::chrono::milliseconds(100), false}}; }
static const auto SIM_DURATION = std::chrono::months{12};
static const int SIM_RUNS = 32768;
"""

HIP_PRELUDE = r"""
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
"""


def _blocks():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        return re.findall(r"```cpp\n(.*?)```", f.read(), re.S)


def _compile(tmp_path, name, src, hip=False):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    p = tmp_path / f"{name}.cpp"
    p.write_text((HIP_PRELUDE if hip else "") + PRELUDE + src)
    cmd = [cxx, "-std=c++20", "-fsyntax-only", "-Wall", "-Wno-unused-variable", "-Wno-unused-result",
           "-I", os.path.join(ROOT, "include"), str(p)]
    if hip:
        cmd[1:1] = ["-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, f"{name}:\n{src}\n{r.stderr}"


def test_doc_has_the_four_snippets():
    assert len(_blocks()) == 4


def test_section2_driver_compiles(tmp_path):
    _compile(tmp_path, "s2_main", _blocks()[0])


def test_section2_large_network_compiles(tmp_path):
    body = "void large(int64_t duration_ms) {\n" + _blocks()[1] + "\n}\n"
    _compile(tmp_path, "s2_large", body)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/include/rccl/rccl.h"), reason="RCCL headers absent")
def test_section3_rank_snippet_compiles(tmp_path):
    body = ("void rank(const msim_config *cfg, int g, uint64_t n_per_rank, uint32_t M, hipStream_t stream,\n"
            "          ncclComm_t comm, std::vector<msim_stats> &stats_total) {\n" + _blocks()[2] + "\n}\n")
    _compile(tmp_path, "s3_rank", body, hip=True)


def test_section3_run_multi_compiles(tmp_path):
    body = "void multi(const msim_config *cfg, uint32_t M) {\n" + _blocks()[3] + "\n}\n"
    _compile(tmp_path, "s3_multi", body)
