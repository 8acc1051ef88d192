"""ICP oracle (oracle/icp_oracle.py) pinned against the reference's own outputs
(tests/golden/icp_golden.npz, made by tests/golden/make_icp_golden.py from
utils/icp.py + sklearn).  CPU only."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import icp_oracle  # noqa: E402

GOLD = np.load(os.path.join(ROOT, "tests", "golden", "icp_golden.npz"))


def _case(name):
    p = f"icp/{name}/"
    return {k[len(p):]: GOLD[k] for k in GOLD.files if k.startswith(p)}


@pytest.mark.parametrize("name", [str(c) for c in GOLD["icp_cases"]])
def test_oracle_icp_matches_reference(name):
    c = _case(name)
    kw = dict(max_iterations=int(c["max_iterations"]), tolerance=float(c["tolerance"]))
    if "init_pose" in c:
        kw["init_pose"] = c["init_pose"]
    T, dist, i = icp_oracle.icp(c["A"], c["B"], **kw)
    assert i == int(c["i"])
    np.testing.assert_allclose(T, c["T"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(dist, c["distances"], rtol=1e-12, atol=1e-15)


def test_oracle_nearest_neighbor_matches_sklearn_golden():
    d, k = icp_oracle.nearest_neighbor(GOLD["nn/src"], GOLD["nn/dst"])
    np.testing.assert_array_equal(k, GOLD["nn/indices"])
    np.testing.assert_allclose(d, GOLD["nn/distances"], rtol=1e-15, atol=0)


@pytest.mark.parametrize("name", [str(c) for c in GOLD["bft_cases"]])
def test_oracle_best_fit_transform_matches_reference(name):
    T, R, t = icp_oracle.best_fit_transform(GOLD[f"bft/{name}/A"], GOLD[f"bft/{name}/B"])
    np.testing.assert_allclose(T, GOLD[f"bft/{name}/T"], rtol=0, atol=1e-12)
    assert np.linalg.det(R) > 0


def test_oracle_align_matches_testnet():
    out = icp_oracle.align(GOLD["align/points"], GOLD["align/fake"])
    np.testing.assert_allclose(out, GOLD["align/out"], rtol=0, atol=1e-6)
