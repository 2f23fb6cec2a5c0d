"""The CPU oracle against its committed fingerprints (tests/golden/)."""
import json
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "oracle_golden.json")))


@pytest.mark.parametrize("fx", GOLDEN, ids=[str(g["case"][:2]) for g in GOLDEN])
def test_oracle_matches_golden(oracle, fx):
    import sys

    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_golden

    got = make_golden.fingerprint(tuple(fx["case"]))
    assert got["input_sha256"] == fx["input_sha256"], "synthetic generator drifted"
    assert got == fx
