"""CPU models of the GPU algorithms (no GPU): tools/dc3_sim.py restates the DC3 sorter's
decomposition (dc3.hip: sample keys, naming, the dummy sample, the mod-0 list taken from the
sorted sample, the merge comparator) and must equal a naive suffix sort."""
import os
import sys

import numpy as np

from tests.helpers import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_dc3_model_matches_naive_suffix_sort():
    import dc3_sim

    rng = np.random.default_rng(7)
    cases = [rng.integers(1, s + 1, n) for n in (1, 2, 3, 4, 5, 6, 7, 50, 301, 1000) for s in (1, 2, 5, 40)]
    cases += [np.array([1 + (c == "b") for c in dc3_sim.fib(n)], np.int64) for n in (10, 233, 1597, 2000)]
    for t in cases:
        assert list(dc3_sim.dc3(t)) == dc3_sim.naive_sa(t), list(t)[:20]
