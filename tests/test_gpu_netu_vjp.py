"""FBSNN.net_u as a differentiable op (nd_BSPDE_case.py:191-221: u and
Du = du/dX with create_graph=True, so a loss on (u, Du) back-propagates into
the network parameters).  The native backward is dbsde_net_u_vjp -- the
loss_grad backward with the caller's cotangents -- on the fused split-bf16
kernels (NAIS-Net 4x110), the fp32 fused width-16 kernels, the fused
width-256 kernels (phase2.hip: FC-Sine [101,256x4,1] and [2,256x4,1], configs
4 and 1) and the per-layer chain (FC 4x256 at D = 20, which has no fused
instance).  Checked against the oracle's autograd (oracle/fbsnn_ref.py
net_u, torch CPU) on the same weights, points and cotangents.  Needs a GPU."""
import numpy as np
import pytest
import torch

from conftest import load_pkg
from oracle import fbsnn_ref as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return load_pkg()


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda:0")


@pytest.mark.parametrize("mode,layers,act,form", [("NAIS-Net", [101] + 4 * [110] + [1], "Sine", 1),
                                                  ("Naisnet", [6] + 4 * [16] + [1], "Tanh", None),
                                                  ("FC", [21] + 4 * [256] + [1], "Sine", 4),
                                                  ("FC", [101] + 4 * [256] + [1], "Sine", 1),
                                                  ("FC", [2] + 4 * [256] + [1], "Sine", 1)],
                         ids=["nais110_x3", "naisnet16", "fc256_chain", "fc256_fused_d100", "fc256_fused_d1"])
def test_net_u_backward_matches_reference_autograd(pkg, dev, mode, layers, act, form):
    """form: the solver.matrix_form bit the case must run on (1 = the fused
    split-bf16 phase kernels, 4 = the split-bf16 per-layer chain)."""
    D = layers[0] - 1
    torch.manual_seed(0)
    m = pkg.BlackScholesBarenblatt(np.ones((1, D)), 1.0, 8, 5, D, layers, mode, act, device=dev)
    if form is not None:
        assert m.solver.matrix_form & form, f"expected matrix_form bit {form}, got {m.solver.matrix_form}"
    oracle = ref.build_model(mode, layers, act)
    ref.set_flat_params(oracle, m.params.cpu().numpy())
    rs = np.random.RandomState(1)
    R = 96
    t = rs.uniform(0.0, 1.0, (R, 1)).astype(np.float32)
    X = (1.0 + 0.3 * rs.normal(size=(R, D))).astype(np.float32)
    gu = rs.normal(size=(R, 1)).astype(np.float32)
    gdu = rs.normal(size=(R, D)).astype(np.float32)

    u, du = m.net_u(t, X)
    assert u.requires_grad and du.requires_grad
    loss = (torch.from_numpy(gu).to(dev) * u).sum() + (torch.from_numpy(gdu).to(dev) * du).sum()
    m.model.zero_grad(set_to_none=True)
    loss.backward()
    named = dict(m.model.named_parameters())
    g_nat = torch.cat([(named[n].grad if named[n].grad is not None else torch.zeros_like(named[n])).reshape(-1)
                       for n in m.model.state_dict()]).cpu().numpy()

    Xr = torch.from_numpy(X).requires_grad_(True)
    ur, dur = ref.net_u(oracle, torch.from_numpy(t), Xr)
    ((torch.from_numpy(gu) * ur).sum() + (torch.from_numpy(gdu) * dur).sum()).backward()
    g_ref, used = ref.flat_grads(oracle)

    np.testing.assert_allclose(u.detach().cpu().numpy(), ur.detach().numpy(), rtol=0,
                               atol=1e-4 * max(1.0, float(np.abs(ur.detach().numpy()).max())))
    np.testing.assert_allclose(du.detach().cpu().numpy(), dur.detach().numpy(), rtol=0,
                               atol=1e-4 * max(1.0, float(np.abs(dur.detach().numpy()).max())))
    scale = float(np.abs(g_ref[used]).max())
    np.testing.assert_allclose(g_nat[used], g_ref[used], rtol=0, atol=2e-4 * scale)
    assert np.all(g_nat[~used] == 0.0)


def test_net_u_without_grad_mode_is_detached(pkg, dev):
    D = 4
    m = pkg.BlackScholesBarenblatt(np.ones((1, D)), 1.0, 8, 5, D, [D + 1] + 4 * [16] + [1], "NAIS-Net", "Sine",
                                   device=dev)
    with torch.no_grad():
        u, du = m.net_u(np.zeros((3, 1), np.float32), np.ones((3, D), np.float32))
    assert not u.requires_grad and not du.requires_grad
