"""The EMD auction's published guarantee, checked against an exact solver.

Parity against the reference's EMD stops at the oracle: the reference's GetMax
is racy (emd_cuda.cu:188-190) and it ships no EMD fixture, so beyond its own
"Verified EMD" invariant (metric/emd/test.py:24-28) nothing of the reference
pins an assignment.  What the reference's algorithm does promise is the
auction's: each winning bid raises its object's price by best - better + eps
(emd_cuda.cu:174-176, 196-215), so every assigned point keeps eps-complementary
slackness -- its object's value (3 - ||x_j - y_k|| - price_k, emd_cuda.cu:146)
is within eps of its best value at the final prices -- and once the auction has
converged to a bijection (metric/emd/README.md: eps "balances the error rate
and the speed of convergence") its total cost sum_j ||x_j - y_a(j)|| is within
n * eps of the optimal assignment's.  Both are checked here, for the CPU oracle
(not gpu) and for the product path at full BASELINE sizes (gpu), against
scipy.optimize.linear_sum_assignment on the same float64 distances.  Settings
use enough iterations to converge before the last one (on the last iteration
every bidder takes its bid unconditionally, emd_cuda.cu:201-205, which the
bijection assertion would catch; the reference's test prints the same count,
|set(assignment)|, metric/emd/test.py:23).  N is a multiple of 1024 as the
reference requires (emd_cuda.cu:246).  Not every documented setting converges:
the README's test-time eps 0.002 with 10000 iterations leaves 2 of 2048 points
per cloud bidding at the last iteration (oracle, seed 5: 4 bidders left from
iteration 8,113 on), so its result is not a bijection -- the reference's own
caveat; that setting is pinned bit-exact against the oracle in test_emd_gpu.py.
"""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment

# float32 values and prices (magnitude < 8): a few ulps of slack on top of eps
SLACK = 1e-5


def _clouds(seed, b, n):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(b, n, 3, generator=g).numpy(), torch.rand(b, n, 3, generator=g).numpy()


def _check_eps_optimal(x1, x2, ass, price, eps):
    """One batch element: bijection, eps-CS at the final prices, and
    OPT <= cost <= OPT + n * eps.  Returns (cost - OPT) / (n * eps)."""
    n = x1.shape[0]
    np.testing.assert_array_equal(np.sort(ass), np.arange(n))  # converged: a bijection
    dif = x1[:, None, :].astype(np.float64) - x2[None, :, :].astype(np.float64)
    dist = np.sqrt((dif * dif).sum(-1))
    val = (3.0 - dist) - price.astype(np.float64)[None, :]
    rows = np.arange(n)
    gap = val.max(1) - val[rows, ass]
    assert gap.max() <= eps + SLACK, f"eps-CS broken: worst gap {gap.max()} > eps {eps}"
    cost = dist[rows, ass].sum()
    r, c = linear_sum_assignment(dist)
    opt = dist[r, c].sum()
    assert cost >= opt - 1e-9 * n
    assert cost <= opt + n * (eps + SLACK), f"cost {cost} above OPT {opt} + n*eps {n * eps}"
    return (cost - opt) / (n * eps)


@pytest.mark.parametrize("b,n,eps,iters,seed", [
    (1, 1024, 0.005, 10000, 20),  # BASELINE config 3's eps, run to convergence
    (2, 1024, 0.05, 3000, 21),    # loss/loss.py:23 training setting
    (1, 1024, 0.002, 10000, 22),  # metric/emd/README.md test-time setting
])
def test_oracle_emd_is_eps_optimal(oracle, b, n, eps, iters, seed):
    a, c = _clouds(seed, b, n)
    _, ass, price, _ = oracle.emd_forward(a, c, eps, iters, with_stats=True)
    for i in range(b):
        _check_eps_optimal(a[i], c[i], ass[i], price[i], eps)


@pytest.mark.gpu
@pytest.mark.parametrize("b,n,eps,iters,seed", [
    (16, 1024, 0.005, 10000, 0),  # BASELINE config 3 (B=16, N=1024, eps 0.005), run to convergence
    (4, 1024, 0.05, 3000, 1),     # loss/loss.py:23 training setting
    (2, 2048, 0.05, 3000, 6),     # metric/emd/test.py:7-11 setting (N=2048, eps 0.05, 3000 iters)
    (1, 4096, 0.005, 10000, 3),   # beyond the LDS-resident state; converges at iteration 7,210 (oracle)
])
def test_emd_forward_is_eps_optimal(cuda, b, n, eps, iters, seed):
    import pcm_hip
    a, c = _clouds(seed, b, n)
    x1, x2 = torch.from_numpy(a).to(cuda), torch.from_numpy(c).to(cuda)
    dist = torch.empty(b, n, device=cuda)
    ass = torch.empty(b, n, dtype=torch.int32, device=cuda)
    price = torch.empty(b, n, device=cuda)
    pcm_hip.emd_forward(x1, x2, eps, iters, dist, ass, price)
    torch.cuda.synchronize()
    ass, price = ass.cpu().numpy(), price.cpu().numpy()
    excess = [_check_eps_optimal(a[i], c[i], ass[i], price[i], eps) for i in range(b)]
    assert max(excess) <= 1.0
