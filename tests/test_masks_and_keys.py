"""CPU: the observability mask tables against a fixture extracted from the reference, and
the jax PRNGKey seed conversion (negative / out-of-range seeds)."""
import json
import os

import numpy as np
import pytest

import pob_np as P

HERE = os.path.dirname(os.path.abspath(__file__))


def test_masks_match_reference_fixture():
    """po_brax/standard_observability_masks.py:5-67, parsed to data by
    tests/golden/make_mask_fixture.py: every dict, every env, every index, same order."""
    from po_brax_amd import standard_observability_masks as M
    fx = json.load(open(os.path.join(HERE, "golden", "observability_masks.json")))["masks"]
    assert set(fx) == {"POSITION", "VELOCITY", "TARGET_POS", "OBJECT_POS", "HEADINGS", "CFRC"}
    for name, table in fx.items():
        ours = getattr(M, name)
        assert set(ours) == set(table), name
        for env, idx in table.items():
            np.testing.assert_array_equal(np.asarray(ours[env]), np.asarray(idx), err_msg=f"{name}[{env}]")


def test_prngkey_seed_conversion():
    """jax.random.PRNGKey with x64 off: the seed goes through np.int64 then int32, key =
    [seed >> 32 (logical, = 0), seed & 0xFFFFFFFF]; seeds outside int64 raise OverflowError.
    In-int32 values follow jax's threefry_seed; the int64 wrap for larger seeds is
    parity-unpinned (no reference fixture holds one)."""
    from po_brax_amd import jumpy
    for seed, want in ((0, [0, 0]), (42, [0, 42]), (-1, [0, 4294967295]), (-7, [0, 4294967289]),
                       (2 ** 31 - 1, [0, 2147483647]), (-(2 ** 31), [0, 2147483648]),
                       (2 ** 31, [0, 2147483648]), (2 ** 40 + 5, [0, 5]), (-(2 ** 31) - 1, [0, 2147483647])):
        assert jumpy.random_prngkey(seed, device="cpu").tolist() == want, seed
        assert P.prngkey(seed).tolist() == want, seed
    for bad in (2 ** 63, -(2 ** 63) - 1, 2 ** 80):
        with pytest.raises(OverflowError):
            jumpy.random_prngkey(bad, device="cpu")
