"""Writes oracle_vectors.npz: per-run (found, stale, best_height) for fixed seeds and configs, produced by
the CPU oracle (oracle/msim_oracle.c, pinned by test_oracle.py against the reference's own KATs). The GPU
parity tests compare against these without re-running the oracle, and test_oracle.py re-derives them to
guard the oracle against regressions. Run: python tests/golden/make_oracle_vectors.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle  # noqa: E402

D = 31_556_952_000
H = [30, 29, 12, 11, 8, 5, 3, 1, 1]
SF = [40, 19, 12, 11, 8, 5, 3, 1, 1]
CONFIGS = {
    "c1_prop10s": (H, [10_000] * 9, [0] * 9),
    "c2_prop100ms": (H, [100] * 9, [0] * 9),
    "default_prop1s": (H, [1_000] * 9, [0] * 9),
    "c3_selfish40_prop1s": (SF, [1_000] * 9, [1] + [0] * 8),
    "c4_selfish49_prop30s": ([49, 10, 12, 11, 8, 5, 3, 1, 1], [30_000] * 9, [1] + [0] * 8),
    "c4_selfish10_prop100ms": ([10, 49, 12, 11, 8, 5, 3, 1, 1], [100] * 9, [1] + [0] * 8),
}
N = 64


def main():
    out = {}
    for name, (p, q, s) in CONFIGS.items():
        f, st, _, _ = pyoracle.run_batch(p, q, s, D, N, 0, 1000, threads=8)
        bh = np.array([pyoracle.run(p, q, s, D, 1000 + 2 * r, 1001 + 2 * r)[2] for r in range(N)], dtype=np.int64)
        out[name + "_found"] = f.astype(np.int64)
        out[name + "_stale"] = st.astype(np.int64)
        out[name + "_best_height"] = bh
        out[name + "_config"] = np.array([p, q, s], dtype=np.int64)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_vectors.npz"), **out)


if __name__ == "__main__":
    main()
