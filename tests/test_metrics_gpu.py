"""GPU parity of the evaluation-metric caller (utils/metrics.py counterpart).

Metrics.get (utils/metrics.py:30-37) -> _get_emd_distance (:49-53: EMD with
eps 0.005, 50 iterations, 100 * mean over clouds of mean(sqrt(dist))) and
_get_chamfer_distance (:56-60: 100 * (mean(dist1) + mean(dist2))), checked
against the CPU oracle on the same clouds; and the testnet.py:57-70 sequence
(ICP-align every prediction to its ground truth, then Metrics.get) against the
ICP oracle (oracle/icp_oracle.py, pinned to the reference's utils/icp.py) plus
the metric oracle.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _clouds(seed, b, n):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(b, n, 3, generator=g), torch.rand(b, n, 3, generator=g)


def _oracle_metrics(oracle, pred, gt):
    """The reference's two reductions on the oracle's outputs (float32 values,
    reduced in float64; the GPU path reduces in float32)."""
    ed, _ = oracle.emd_forward(pred, gt, 0.005, 50)
    emd = float(np.sqrt(ed.astype(np.float64)).mean(1).mean()) * 100
    d1, d2, _, _ = oracle.chamfer_forward(pred, gt)
    cd = (float(d1.astype(np.float64).mean()) + float(d2.astype(np.float64).mean())) * 100
    return emd, cd


@pytest.mark.parametrize("b,n,seed", [(4, 1024, 0), (32, 1024, 1), (2, 2048, 2)])
def test_metrics_get_matches_oracle(cuda, oracle, b, n, seed):
    import metrics
    a, c = _clouds(seed, b, n)
    got = metrics.Metrics.get(a.to(cuda), c.to(cuda))
    assert metrics.Metrics.names() == ["EMD_distance", "ChamferDistance"]
    emd, cd = _oracle_metrics(oracle, a.numpy(), c.numpy())
    assert abs(got[0] - emd) <= 2e-5 * abs(emd)
    assert abs(got[1] - cd) <= 2e-5 * abs(cd)


def test_metrics_per_call_values_are_the_oracle_outputs(cuda, oracle):
    # the two metric modules' raw outputs equal the oracle's bit for bit
    import metrics
    a, c = _clouds(3, 4, 1024)
    emd_mod = metrics.Metrics.ITEMS[0]['eval_object']
    cd_mod = metrics.Metrics.ITEMS[1]['eval_object']
    dist, ass = emd_mod(a.to(cuda), c.to(cuda), eps=0.005, iters=50)
    rd, ra = oracle.emd_forward(a.numpy(), c.numpy(), 0.005, 50)
    np.testing.assert_array_equal(ass.cpu().numpy(), ra)
    np.testing.assert_array_equal(dist.cpu().numpy().view(np.int32), rd.view(np.int32))
    d1, d2, i1, i2 = cd_mod(a.to(cuda), c.to(cuda))
    r1, r2, j1, j2 = oracle.chamfer_forward(a.numpy(), c.numpy())
    np.testing.assert_array_equal(i1.cpu().numpy(), j1)
    np.testing.assert_array_equal(d2.cpu().numpy().view(np.int32), r2.view(np.int32))


def test_metrics_disabled_item_and_records(cuda):
    import metrics
    a, c = _clouds(4, 2, 1024)
    item = metrics.Metrics.ITEMS[0]
    item['enabled'] = False
    try:
        vals = metrics.Metrics.get(a.to(cuda), c.to(cuda))
        assert len(vals) == 1 and metrics.Metrics.names() == ["ChamferDistance"]
    finally:
        item['enabled'] = True
    m = metrics.Metrics('ChamferDistance', metrics.Metrics.get(a.to(cuda), c.to(cuda)))
    worse = metrics.Metrics('ChamferDistance', {'ChamferDistance': 1e9, 'EMD_distance': 1e9})
    assert m.better_than(worse) and not worse.better_than(m) and m.better_than(None)


def test_testnet_sequence_icp_aligned_metrics(cuda, oracle):
    # testnet.py:57-70 for a batch: T = icp(points[k], fake[k], 1e-10, 1024);
    # fake_k @ T[:3,:3] - T[:3,3] as float32; Metrics.get(aligned, points)
    import icp as icp_mod
    import icp_oracle
    import metrics
    g = torch.Generator().manual_seed(5)
    points = torch.rand(3, 1024, 3, generator=g)
    rot = torch.tensor([[0.995, -0.0998, 0.0], [0.0998, 0.995, 0.0], [0.0, 0.0, 1.0]])
    fake = (points @ rot + 0.01 * torch.randn(3, 1024, 3, generator=g) + 0.02).contiguous()
    aligned = icp_mod.align_predictions(fake.to(cuda), points.to(cuda))
    got = metrics.Metrics.get(aligned, points.to(cuda))
    # the alignment against the ICP oracle (float64 transforms; the float32
    # aligned clouds may differ in the last ulp)
    ref_aligned = []
    for k in range(3):
        T, _, _ = icp_oracle.icp(points[k].double().numpy(), fake[k].double().numpy(), tolerance=1e-10,
                                 max_iterations=1024)
        ref_aligned.append(fake[k].double().numpy() @ T[:3, :3] - T[:3, 3])
    ref_aligned = np.array(ref_aligned).astype(np.float32)
    np.testing.assert_allclose(aligned.cpu().numpy(), ref_aligned, rtol=0, atol=2e-6)
    # the metrics on the GPU-aligned clouds: the oracle's values on the same clouds
    emd, cd = _oracle_metrics(oracle, aligned.cpu().numpy(), points.numpy())
    assert abs(got[0] - emd) <= 2e-5 * abs(emd)
    assert abs(got[1] - cd) <= 2e-5 * abs(cd)
    # and close to the values on the oracle-aligned clouds (an ulp in an input
    # may move an auction assignment, so this one is a tolerance)
    emd_r, cd_r = _oracle_metrics(oracle, ref_aligned, points.numpy())
    assert abs(got[0] - emd_r) <= 1e-3 * abs(emd_r)
    assert abs(got[1] - cd_r) <= 1e-4 * abs(cd_r)
