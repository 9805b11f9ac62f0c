"""CPU tests of the spec's elementary functions in the oracle (the HIP kernels spell the same
operations; their bit-exact agreement is covered by the GPU step / reset parity tests).

* atan2f: branch-free octant reduction + degree-7 minimax polynomial:
  <= 4 ulp (plus 1e-45 absolute) against float64 arctan2 over the plane, exact special cases.
* substep quaternion normalisation: series 1 - e/2 + 3e^2/8 - 5e^3/16 in e = |q|^2 - 1 for
  |e| <= 2^-6, 1 / sqrt(|q|^2) beyond (both within 2 ulp of the exact unit quaternion).
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import orc  # noqa: E402


def _ulp_err(got, ref):
    ref32 = np.abs(ref).astype(np.float32)
    return np.abs(got.astype(np.float64) - ref) / np.spacing(np.maximum(ref32, np.float32(1e-30))).astype(np.float64)


def test_atan2_accuracy_over_the_plane():
    rng = np.random.default_rng(0)
    n = 400_000
    ang = rng.uniform(-np.pi, np.pi, n)
    rad = np.exp(rng.uniform(-20, 20, n))
    y = (rad * np.sin(ang)).astype(np.float32)
    x = (rad * np.cos(ang)).astype(np.float32)
    got = orc.math_check(0, y, x)
    ref = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    assert _ulp_err(got, ref).max() <= 4.0


def test_atan2_octant_boundaries_and_specials():
    # |x| == |y|, axis directions, tiny / huge magnitudes, signed zeros, NaN
    v = np.float32([1.0, 3.0e-38, 1.5e38, 0.7071068])
    ys, xs = [], []
    for s in v:
        for a, b in ((s, s), (s, -s), (-s, s), (-s, -s), (s, 0.0), (-s, 0.0), (0.0, s), (0.0, -s)):
            ys.append(a)
            xs.append(b)
    y = np.float32(ys)
    x = np.float32(xs)
    got = orc.math_check(0, y, x)
    ref = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    assert _ulp_err(got, ref).max() <= 4.0
    sp = orc.math_check(0, np.float32([0.0, -0.0, 0.0, -0.0, np.nan, 1.0]), np.float32([0.0, 0.0, -1.0, -1.0, 1.0, np.nan]))
    assert sp[0] == 0.0 and sp[1] == 0.0
    assert sp[2] == np.float32(np.pi) and sp[3] == -np.float32(np.pi)
    assert np.isnan(sp[4]) and np.isnan(sp[5])


@pytest.mark.parametrize("emax", [2.0 ** -6, 2.0 ** -2])
def test_substep_normalisation(emax):
    rng = np.random.default_rng(1)
    n = 200_000
    u = rng.normal(size=(n, 4))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    e = rng.uniform(-emax, emax, n)  # |q|^2 = 1 + e
    q = (u * np.sqrt(1.0 + e)[:, None]).astype(np.float32)
    got = orc.math_check(1, q).astype(np.float64)
    ref = q.astype(np.float64) / np.linalg.norm(q.astype(np.float64), axis=1, keepdims=True)
    err = np.abs(got - ref).max(1)
    assert err.max() < 3 * 2.0 ** -24  # within a few ulp of the exact unit quaternion
    assert np.abs(np.linalg.norm(got, axis=1) - 1.0).max() < 4 * 2.0 ** -24
