"""Product-side initialisation parity.

Under np.random.seed(42) the skge_amd model constructors must give the
reference's initial tables -- drawn by the reference's own constructors in
tools/gen_golden.py (tests/golden/init_quirks.npz) -- rounded to fp32:

* TransE: E init_nunif then row-normalised (skge/transe.py:14-23,
  skge/param.py:161-167 with idx None), R init_nunif, E drawn before R;
* HolE: E init_nunif then the column-wise normless1 quirk (skge/hole.py:16,
  skge/param.py:170-174: M[None] sums over rows), R init_nunif;
* RESCAL: E init_nunif (no post), every W slice its own init_nunif((d, d))
  draw (skge/param.py:62-64).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _z():
    return np.load(os.path.join(GOLDEN, "init_quirks.npz"))


def _f32(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def test_transe_constructor_matches_reference_init():
    import skge_amd as S
    z = _z()
    np.random.seed(42)
    m = S.TransE((50, 50, 4), 8)
    assert m.E.data.dtype.is_floating_point and m.E.data.is_cuda
    np.testing.assert_array_equal(m.E.data.cpu().numpy(), _f32(z["transe_E"]))
    np.testing.assert_array_equal(m.R.data.cpu().numpy(), _f32(z["transe_R"]))
    # unit rows after the init projection (to fp32 rounding)
    np.testing.assert_allclose(np.linalg.norm(m.E.data.cpu().numpy().astype(np.float64), axis=1),
                               1.0, atol=1e-6)


def test_hole_constructor_matches_reference_column_quirk():
    import skge_amd as S
    z = _z()
    np.random.seed(42)
    m = S.HolE((50, 50, 4), 8)
    E = m.E.data.cpu().numpy()
    np.testing.assert_array_equal(E, _f32(z["hole_E"]))
    np.testing.assert_array_equal(m.R.data.cpu().numpy(), _f32(z["hole_R"]))
    # the quirk: columns, not rows, were divided by max(sum of squares, 1)
    assert not np.allclose(np.linalg.norm(E.astype(np.float64), axis=1), 1.0, atol=1e-3)


def test_rescal_constructor_matches_reference_slices():
    import skge_amd as S
    z = _z()
    np.random.seed(42)
    m = S.RESCAL((50, 50, 3), 4)
    np.testing.assert_array_equal(m.E.data.cpu().numpy(), _f32(z["rescal_E"]))
    np.testing.assert_array_equal(m.W.data.cpu().numpy(), _f32(z["rescal_W"]))


def test_constructor_draw_order_continues_the_global_stream():
    """Two models built back to back draw from one global stream (E, R of the
    first, then the second's): the second equals the reference's tables drawn
    after the first's."""
    import skge_amd as S
    from oracle import skge_oracle as O
    np.random.seed(42)
    S.TransE((50, 50, 4), 8)
    m2 = S.TransE((30, 30, 2), 8)
    np.random.seed(42)
    O.init_nunif((50, 8))
    O.init_nunif((4, 8))
    E2 = O.normalize(O.init_nunif((30, 8)), None)
    R2 = O.init_nunif((2, 8))
    np.testing.assert_array_equal(m2.E.data.cpu().numpy(), E2.astype(np.float32))
    np.testing.assert_array_equal(m2.R.data.cpu().numpy(), R2.astype(np.float32))
