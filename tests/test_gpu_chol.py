"""Dataflow tile Cholesky (ba_kernels.hip chol_dataflow_kernel) vs numpy on
random SPD systems: sizes around the 64-tile boundaries, the rhs row in its
own row block (n % 64 == 0), a single tile, and the not-SPD path (dx = 0)."""
import numpy as np
import pytest
import torch

from gpu_util import host

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _spd(n, rng, cond=1e4):
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    ev = np.geomspace(1.0, cond, n)
    return (Q * ev) @ Q.T


@pytest.mark.parametrize("n", [6, 48, 63, 64, 65, 127, 128, 130, 300, 512, 700, 1530])
def test_dense_spd_solve_matches_numpy(n):
    import droid_backends
    rng = np.random.default_rng(n)
    A = _spd(n, rng)
    b = rng.normal(size=n)
    lm, ep = 1e-4, 0.1
    Ad = A + np.diag(ep + lm * np.diag(A))
    ref = np.linalg.solve(Ad, b)
    dx, failed = droid_backends.dense_spd_solve(torch.tensor(A, device=DEV), torch.tensor(b, device=DEV), lm, ep)
    assert not failed
    np.testing.assert_allclose(host(dx).astype(np.float64), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())


def test_dense_spd_solve_repeatable():
    import droid_backends
    rng = np.random.default_rng(7)
    A = torch.tensor(_spd(700, rng), device=DEV)
    b = torch.tensor(rng.normal(size=700), device=DEV)
    outs = [host(droid_backends.dense_spd_solve(A, b, 1e-4, 0.1)[0]) for _ in range(3)]
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])   # fixed reduction order


def test_not_spd_gives_zero_dx():
    import droid_backends
    rng = np.random.default_rng(3)
    A = _spd(200, rng)
    A[150, 150] = -1e6
    dx, failed = droid_backends.dense_spd_solve(torch.tensor(A, device=DEV), torch.tensor(rng.normal(size=200), device=DEV))
    assert failed
    assert np.all(host(dx) == 0)
