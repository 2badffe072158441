"""The device-mode generator's CPU restatement (oracle/philox.py), pinned by the
Random123 known-answer vectors for Philox4x32-10 (kat_vectors of the Random123
distribution, Salmon et al. SC'11) and by distributional / structural checks of
the increments and the time grid.  CPU only."""
import numpy as np
import pytest

from oracle import philox as ph

# (counter c0..c3, key k0 k1) -> output, Random123 kat_vectors "philox4x32 10"
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox4x32_10_known_answers(ctr, key, expect):
    out = ph.philox4x32_10(ctr, key)
    assert tuple(int(v) for v in out) == expect


def test_normals_are_standard():
    z = ph.normal4(7, 0, np.arange(4096)[:, None], np.arange(8)[None, :], 3).reshape(-1)
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1.0) < 0.02


def test_increments_shard_by_global_path():
    """Paths [path0, path0 + M) of a rank == the same rows of one device's draw."""
    full = ph.increments(3, 5, 0, 8, 9, 4, 1.0)
    part = ph.increments(3, 5, 4, 4, 9, 4, 1.0)
    np.testing.assert_array_equal(full[4:], part)


def test_correlated_increments_apply_L():
    rs = np.random.RandomState(0)
    A = rs.normal(size=(5, 5))
    L = np.linalg.cholesky(A @ A.T + 5 * np.eye(5))
    dw = ph.increments(1, 0, 0, 6, 7, 5, 1.0)
    dwc = ph.increments(1, 0, 0, 6, 7, 5, 1.0, L=L)
    np.testing.assert_allclose(dwc, np.einsum("ij,mnj->mni", L, dw.astype(np.float64)), rtol=1e-6, atol=1e-6)


def test_time_grid_is_the_reference_cumsum():
    """DeepBSDE.py:250-258: cumsum of dt = T/N in float64, cast to float32."""
    N, T = 50, 1.0
    Dt = np.zeros((1, N + 1, 1))
    Dt[:, 1:, :] = T / N
    ref = np.cumsum(Dt, axis=1).astype(np.float32)[0, :, 0]
    np.testing.assert_array_equal(ph.time_grid(N, T), ref)


def test_brownian_W_is_cumsum_of_increments():
    dw = ph.increments(2, 0, 0, 3, 6, 2, 1.0)
    W = ph.brownian_W(dw)
    assert np.all(W[:, 0] == 0)
    np.testing.assert_allclose(np.diff(W.astype(np.float64), axis=1), dw, rtol=0, atol=1e-6)


def test_heston_rollout_one_asset_matches_the_reference_restatement():
    """The k = 1 NumPy Heston path equals oracle/fbsnn_ref's torch restatement
    of heston_dnnpde.py:629-642 bit for bit on the same increments."""
    import torch
    from oracle import fbsnn_ref as fr
    dw = ph.increments(4, 0, 0, 5, 6, 1, 1.0)
    W = ph.brownian_W(dw)
    X, _ = ph.heston_rollout(np.array([[1.0, 0.2]]), np.diff(W, axis=1), 1.0)
    t = torch.from_numpy(np.broadcast_to(ph.time_grid(6, 1.0)[None, :, None], (5, 7, 1)).copy())
    model = fr.build_heston_model("FC", [2, 4, 4, 1], "Sine", 1)
    h = fr.Heston(k=1)
    xi = torch.tensor([[1.0]], requires_grad=True)
    _, Xr, _, _ = fr.heston_loss_function(model, h, t, torch.from_numpy(W), xi, 5)
    np.testing.assert_array_equal(X, Xr.detach().numpy())
