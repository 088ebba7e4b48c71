"""Oracle ranking (oracle/skge_oracle.py filtered_ranks) against the positions
the reference's own evaluators produced (tests/golden/eval_*.npz, made by
tools/gen_golden_eval.py)."""
import os

import numpy as np
import pytest

from oracle import skge_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("model", ["transe", "hole"])
def test_oracle_ranks_match_reference_positions(model):
    z = np.load(os.path.join(GOLD, "eval_%s.npz" % model))
    got = O.filtered_ranks(model, z["E"], z["R"], z["queries"], z["known"])
    np.testing.assert_array_equal(got[:, 0], z["tail_raw"])
    np.testing.assert_array_equal(got[:, 1], z["tail_filt"])
    np.testing.assert_array_equal(got[:, 2], z["head_raw"])
    np.testing.assert_array_equal(got[:, 3], z["head_filt"])


def test_compute_scores():
    mrr, mean, hits = O.compute_scores([1, 2, 10, 20])
    assert mrr == pytest.approx((1 + 0.5 + 0.1 + 0.05) / 4)
    assert mean == pytest.approx(8.25)
    assert hits == pytest.approx(75.0)
