"""CPU: the oracle reproduces the committed fixtures (tests/golden/*.npz) bit-for-bit.

The fixtures hold seeded problems (incl. REFINE_ITER + APD anchors + geometric consistency + SA mask)
and the outputs the oracle produced when they were generated (tests/golden/make_golden.py). This pins
the oracle against silent drift; the GPU tier checks the HIP path against the same files.
"""
import os

import pytest

import golden_io
import oracle_lib

FIXTURES = golden_io.fixtures()


@pytest.fixture(scope="module")
def oracle():
    return oracle_lib.load()


def test_fixtures_present():
    names = {os.path.basename(f) for f in FIXTURES}
    assert {"first_n4.npz", "refine_iter_apd_geom_sa.npz"} <= names


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(f) for f in FIXTURES])
def test_oracle_matches_fixture(path, oracle):
    arr, expected = golden_io.load(path)
    got = oracle_lib.run(oracle, arr)
    d = golden_io.diff(expected, got)
    assert all(v == 0 for v in d.values()), d
