"""tools/line_model.py (the full-resolution cache-line model DESIGN's verdict
item 3 cites) on a small pixel ring: the line counts per sample fall as the
reuse window widens (one instruction >= one iteration >= W chunks >= the
whole image), the cell layout never needs more than one line per sample, and
a narrow cloud reuses more than a uniform one."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import line_model as lm  # noqa: E402


def test_line_model_orders_its_windows():
    rng = np.random.default_rng(0)
    for layout in ("cells", "ypair"):
        narrow = lm.model(rng, 1.5, layout, 1, ru=20, nrot=32)
        wide = lm.model(rng, None, layout, 1, ru=20, nrot=32)
        for r in (narrow, wide):
            seq = [r["window_1_chunks"], r["window_4_chunks"], r["window_16_chunks"],
                   r["window_64_chunks"], r["whole_image"]]
            assert all(a >= b - 1e-12 for a, b in zip(seq, seq[1:])), seq
            assert r["window_1_chunks"] <= r["per_instruction"] + 1e-12
            assert r["whole_image"] > 0
        if layout == "cells":
            assert wide["per_instruction"] <= 1.0 + 1e-12
        assert narrow["whole_image"] < wide["whole_image"]
