"""Round-4 cases on the HIP path (needs an MI355X):

  * loss_function's loss is connected to the model parameters: a caller's
    own loss.backward() (DeepBSDE.py:278-279) fills .grad with the native
    gradient, scaled by the incoming cotangent, and leaves the never-used
    NAIS-Net input_layers[K] at None;
  * the differentiable net_u on the Heston problem, whose u = max(net, 0)
    clamp masks the backward (heston_dnnpde.py:560-579), at points on both
    sides of the clamp, against the oracle's autograd;
  * the correlated device rollout at config 3's full shape (M = 4096,
    D = 100, N = 50): device increments against the oracle's L (sqrt(dt) z)
    and X bit-exact against the oracle rollout of those increments;
  * the fused optimizer update (dbsde_train_step) with the next batch's
    rollout prefetched beside it, against separate launches (the projection
    adjoint reads a snapshot of W, not the parameters being updated).

Config 1 (the 1-D call, FC-Sine [2,256x4,1], Q3 active) runs through
tests/test_gpu_parity.py::test_loss_grad_matches_reference on the reference
fixtures g1_w256_oned_call_FC_Sine_M16_N5 and _M256_N50 (the full shape)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_pkg
from oracle import fbsnn_ref as fr
from oracle import philox as ph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    return load_pkg()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


def _load(name):
    z = np.load(os.path.join(GOLDEN, name))
    return {k: z[k] for k in z.files}


def _flat_grad(m):
    named = dict(m.model.named_parameters())
    return named, torch.cat([(named[n].grad if named[n].grad is not None else torch.zeros_like(named[n])).reshape(-1)
                             for n in m.model.state_dict()])


@pytest.mark.parametrize("fixture,cls,mode", [("g1_w110_deep_bsb_NAIS-Net_ReLU.npz", "BlackScholesBarenblatt",
                                               "NAIS-Net"),
                                              ("g1_w256_oned_call_FC_Sine_M16_N5.npz", "CallOption1D", "FC")])
def test_loss_function_backward_fills_grad(pkg, dev, fixture, cls, mode):
    g = _load(fixture)
    layers = [int(v) for v in g["layers"]]
    D, M, N = layers[0] - 1, int(g["M"]), int(g["N"])
    C = getattr(pkg, cls)
    if cls == "BlackScholesBarenblatt":
        m = C(g["Xi"], 1.0, M, N, D, layers, mode, str(g["activation"]), device=dev)
    else:
        m = C(g["Xi"], 1.0, M, N, D, 5.0, layers, mode, str(g["activation"]), device=dev)
    m.params.copy_(torch.from_numpy(g["params"]).to(dev))
    t = torch.from_numpy(g["t"]).to(dev)
    W = torch.from_numpy(g["W"]).to(dev)
    m.model.zero_grad(set_to_none=True)
    loss, X, Y, _ = m.loss_function(t, W, m.Xi)
    assert loss.requires_grad and not X.requires_grad and not Y.requires_grad
    (3.0 * loss).backward()
    named, g_bwd = _flat_grad(m)
    # the native gradient of the same batch, through the solver directly
    grad = torch.empty_like(m.params)
    m.solver.loss_grad(m.params, M, N, m._xi_rows(m.Xi, M), t=t.reshape(M, N + 1).contiguous(), W=W.contiguous(),
                       grad=grad, loss=torch.empty(1, device=dev))
    torch.cuda.synchronize()
    torch.testing.assert_close(g_bwd, 3.0 * grad, rtol=0, atol=0)
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-4)
    used = g["used"]
    ref = g["grad"]
    np.testing.assert_allclose(g_bwd.cpu().numpy()[used] / 3.0, ref[used], rtol=0, atol=2e-4 * np.abs(ref).max())
    # parameters no output depends on keep grad None, as under torch autograd
    for name, p in named.items():
        if name.startswith("input_layers.") and mode == "NAIS-Net" and name.split(".")[1] == str(len(layers) - 3):
            assert p.grad is None, name
    with torch.no_grad():
        l2 = m.loss_function(t, W, m.Xi)[0]
    assert not l2.requires_grad


@pytest.mark.parametrize("k,layers_h,act", [(1, 4 * [16], "Tanh"), (3, 4 * [110], "Sine"), (50, 4 * [110], "Sine")],
                         ids=["k1_w16_fused_fp32", "k3_w110_chain", "k50_w110_fused_x3"])
def test_heston_net_u_backward_through_the_clamp(pkg, dev, k, layers_h, act):
    """heston_dnnpde.py:560-579: u = max(net, 0); the backward of (u, Du)
    passes only where net >= 0.  The output bias is set to the median of the
    unclamped outputs, so about half of the points are clamped."""
    torch.manual_seed(40 + k)
    m = pkg.HestonFBSNN(np.ones((1, k)), 1.0, 8, 5, k, None, [2] + layers_h + [1], "Naisnet", act, device=dev)
    D = 2 * k
    oracle = fr.build_heston_model("Naisnet", [2] + layers_h + [1], act, k)
    rs = np.random.RandomState(5)
    R = 96
    t = rs.uniform(0.0, 1.0, (R, 1)).astype(np.float32)
    X = np.concatenate([1.0 + 0.3 * rs.normal(size=(R, k)), 0.2 + 0.05 * rs.uniform(size=(R, k))], 1).astype(np.float32)
    # centre the output on the median raw value: half the rows clamp
    fr.set_flat_params(oracle, m.params.cpu().numpy())
    with torch.no_grad():
        raw = oracle(torch.cat([torch.from_numpy(t), torch.from_numpy(X)], 1)).numpy().ravel()
    names = list(m.model.state_dict())
    out_bias = names[-1]
    off = sum(v.numel() for v in list(m.model.state_dict().values())[:-1])
    m.params[off] -= float(np.median(raw))
    fr.set_flat_params(oracle, m.params.cpu().numpy())
    assert out_bias.endswith("bias")
    gu = rs.normal(size=(R, 1)).astype(np.float32)
    gdu = rs.normal(size=(R, D)).astype(np.float32)
    u, du = m.net_u(t, X)
    loss = (torch.from_numpy(gu).to(dev) * u).sum() + (torch.from_numpy(gdu).to(dev) * du).sum()
    m.model.zero_grad(set_to_none=True)
    loss.backward()
    _, g_nat = _flat_grad(m)
    Xr = torch.from_numpy(X).requires_grad_(True)
    ur, dur = fr.heston_net_u(oracle, torch.from_numpy(t), Xr)
    nclamp = int((ur.detach().numpy() == 0).sum())
    assert 0.25 * R < nclamp < 0.75 * R, nclamp
    ((torch.from_numpy(gu) * ur).sum() + (torch.from_numpy(gdu) * dur).sum()).backward()
    g_ref, used = fr.flat_grads(oracle)
    np.testing.assert_allclose(u.detach().cpu().numpy(), ur.detach().numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(du.detach().cpu().numpy(), dur.detach().numpy(), rtol=0,
                               atol=1e-4 * max(1.0, float(np.abs(dur.detach().numpy()).max())))
    g_nat = g_nat.cpu().numpy()
    scale = float(np.abs(g_ref[used]).max())
    np.testing.assert_allclose(g_nat[used], g_ref[used], rtol=0, atol=2e-4 * scale)


def test_correlated_device_rollout_at_config3_shape(pkg, dev):
    """with_corr...py:339-341 at config 3's shape (M = 4096, D = 100, N = 50,
    the Q10 correlation recipe): the device increments L (sqrt(dt) z) against
    the oracle's (fp32 summation order differs: 2e-6 relative per term), and X
    bit-exact against the oracle's rollout of the device increments."""
    D, M, N = 100, 4096, 50
    np.random.seed(3)
    L = np.linalg.cholesky(pkg.FBSNN._random_corr(D, False)).astype(np.float32)
    spec = pkg.ProblemSpec(mu_a=0.05, sig_a=0.20, phi_r=0.05, phi_c=0.0, g="call_mean", strike=1.0)
    s = pkg.NativeSolver("Naisnet", [D + 1] + 4 * [110] + [1], "ReLU", spec, 1.0, dev)
    s.set_corr(L)
    _, dW = s.brownian(M, N, seed=17, increments=True)
    dW = dW.cpu().numpy()
    ref = ph.increments(17, 0, 0, M, N, D, 1.0, L=L)
    # fp32 dot products in another order (|err| <= D 2^-24 sum_j |L_ij xi_j|)
    # plus the device normals' 2e-6 tolerance (tests/test_gpu_device_rng.py)
    bound = np.einsum("ij,mnj->mni", np.abs(L), np.abs(ph.increments(17, 0, 0, M, N, D, 1.0)))
    bound = 2e-6 * np.sqrt(D) * bound + 4e-6 * np.sqrt(1.0 / N) * np.abs(L).sum(1)
    assert np.all(np.abs(dW - ref) <= bound)
    Xi = np.ones((1, D))
    X = torch.empty(M * (N + 1) * D, device=dev)
    s.loss_grad(torch.zeros(s.nparams, device=dev), M, N, torch.ones(D, device=dev), seed=17, X=X,
                loss=torch.empty(1, device=dev))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(X.cpu().numpy().reshape(M, N + 1, D), ph.rollout(Xi, dW, 1.0, 0.05, 0.2, 0.0))


def test_fused_update_with_a_prefetched_rollout_beside_it(pkg, dev):
    """dbsde_train_step with the optimizer update folded into the finalize and
    the projection adjoint, while the next batch's rollout runs on another
    stream (it takes CUs, so the finalize / adjoint blocks are not all
    resident together): bit-identical to loss_grad + optimizer_step."""
    g = _load("g2_north_star.npz")
    layers = [int(v) for v in g["layers"]]
    D = layers[0] - 1

    def model():
        m = pkg.BlackScholesBarenblatt(g["Xi"], 1.0, 1024, 50, D, layers, "NAIS-Net", "Sine", device=dev)
        m.params.copy_(torch.from_numpy(g["params"]).to(dev))
        return m

    a, b = model(), model()
    oa, ob = a.new_optimizer_state("Adam", 1e-3), b.new_optimizer_state("Adam", 1e-3)
    for s in range(4):
        a.device_step(oa, seed=s, next_seed=s + 1)                         # fused + prefetch
        b.solver.loss_grad(b.params, b.M, b.N, b._device_xi(0, b.M), seed=s, grad=b.grad, loss=b._gradbuf[-1:])
        b._update(ob)
    torch.cuda.synchronize()
    for x, y in ((a.params, b.params), (oa["m"], ob["m"]), (oa["v"], ob["v"])):
        torch.testing.assert_close(x, y, rtol=0, atol=0)


@pytest.mark.parametrize("name", ["g1_w256_hjb_FC_Sine_N20.npz", "g1_w256_oned_call_FC_Sine_M16_N5.npz",
                                  "g1_w256_oned_call_FC_Sine_M256_N50.npz"])
def test_width256_fused_kernels_match_reference(pkg, dev, name):
    """Config 4's FC-Sine [101,256x4,1] (hjb_implement.py:590-604) and config
    1's FC-Sine [2,256x4,1] (call_option_1d.py) on the fused width-256 phase
    kernels (phase2.hip, one 16-row tile per wave, adot through memory; the
    default, DBSDE_W256=1 made explicit) against the reference fixtures,
    tolerances as test_gpu_parity."""
    from test_gpu_parity import make_solver
    g = _load(name)
    old = os.environ.get("DBSDE_W256")
    os.environ["DBSDE_W256"] = "1"
    try:
        s = make_solver(pkg, dev, g)
    finally:
        if old is None:
            del os.environ["DBSDE_W256"]
        else:
            os.environ["DBSDE_W256"] = old
    assert s.matrix_form & 1 and not s.matrix_form & 4, "expected the fused split-bf16 kernels"
    layers = [int(v) for v in g["layers"]]
    D, M, N = layers[0] - 1, int(g["M"]), int(g["N"])
    params = torch.from_numpy(g["params"]).to(dev)
    out = dict(loss=torch.empty(1, device=dev), X=torch.empty(M * (N + 1) * D, device=dev),
               Y=torch.empty(M * (N + 1), device=dev), Z=torch.empty(M * (N + 1) * D, device=dev))
    grad = torch.empty_like(params)
    s.loss_grad(params, M, N, torch.from_numpy(g["Xi"]).to(dev).contiguous(),
                t=torch.from_numpy(g["t"]).to(dev).reshape(M, N + 1).contiguous(),
                W=torch.from_numpy(g["W"]).to(dev).contiguous(), grad=grad, **out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["X"].cpu().numpy().reshape(M, N + 1, D), g["X"])
    np.testing.assert_allclose(float(out["loss"]), float(g["loss"]), rtol=1e-4)
    Y = out["Y"].cpu().numpy().reshape(M, N + 1, 1)
    np.testing.assert_allclose(Y, g["Y"], rtol=0, atol=1e-4 * max(1.0, np.abs(g["Y"]).max()))
    if "Z" in g:
        Z = out["Z"].cpu().numpy().reshape(M, N + 1, D)
        np.testing.assert_allclose(Z, g["Z"], rtol=0, atol=1e-4 * max(1.0, np.abs(g["Z"]).max()))
    used = g["used"]
    r = grad.cpu().numpy()
    np.testing.assert_allclose(r[used], g["grad"][used], rtol=0, atol=2e-4 * np.abs(g["grad"]).max())


@pytest.mark.parametrize("M", [128, 1024])
def test_phase_chunk_count_does_not_change_the_step(pkg, dev, M):
    """The phase pipeline's path chunks (DBSDE_CHUNKS; default by occupancy:
    one chunk when a phase launch fits the chip's workgroup slots, M = 128,
    else two, M = 1024) only reorder independent rows: loss and gradient are
    bit-identical for 1, 2, 4 (weight-gradient slices piped behind each
    chunk) and the default."""
    g = _load("g2_north_star.npz")
    layers = [int(v) for v in g["layers"]]
    D = layers[0] - 1
    res = {}
    old = os.environ.get("DBSDE_CHUNKS")
    try:
        for ch in ("1", "2", "4", None):
            if ch is None:
                os.environ.pop("DBSDE_CHUNKS", None)
            else:
                os.environ["DBSDE_CHUNKS"] = ch
            m = pkg.BlackScholesBarenblatt(g["Xi"], 1.0, M, 50, D, layers, "NAIS-Net", "Sine", device=dev)
            m.params.copy_(torch.from_numpy(g["params"]).to(dev))
            loss = torch.empty(1, device=dev)
            m.solver.loss_grad(m.params, M, 50, m._device_xi(0, M), seed=5, grad=m.grad, loss=loss)
            torch.cuda.synchronize()
            res[ch] = (loss.cpu().clone(), m.grad.cpu().clone())
    finally:
        if old is None:
            os.environ.pop("DBSDE_CHUNKS", None)
        else:
            os.environ["DBSDE_CHUNKS"] = old
    for ch in ("2", "4", None):
        torch.testing.assert_close(res[ch][0], res["1"][0], rtol=0, atol=0)
        torch.testing.assert_close(res[ch][1], res["1"][1], rtol=0, atol=0)


def test_weight_gradient_splits_follow_the_batch(pkg, dev):
    """The chain / width-256 weight-gradient tiles split the rows per batch
    (at least 16 32-row steps per split) and the finalize sums exactly the
    splits written: a step at a small batch after one at a large batch on the
    same context gives the fresh context's gradient bit for bit (no partial
    slab of the larger batch leaks in)."""
    from test_gpu_parity import make_solver
    g = _load("g1_w256_hjb_FC_Sine_N20.npz")
    layers = [int(v) for v in g["layers"]]
    D, M, N = layers[0] - 1, int(g["M"]), int(g["N"])
    params = torch.from_numpy(g["params"]).to(dev)
    xi = torch.from_numpy(g["Xi"]).to(dev).contiguous()

    def small(s):
        grad, loss = torch.empty_like(params), torch.empty(1, device=dev)
        s.loss_grad(params, M, N, xi, t=torch.from_numpy(g["t"]).to(dev).reshape(M, N + 1).contiguous(),
                    W=torch.from_numpy(g["W"]).to(dev).contiguous(), grad=grad, loss=loss)
        torch.cuda.synchronize()
        return grad.cpu(), loss.cpu()

    a = make_solver(pkg, dev, g)
    big = 2048
    gb, lb = torch.empty_like(params), torch.empty(1, device=dev)
    a.loss_grad(params, big, N, xi, seed=3, grad=gb, loss=lb)
    ga, la = small(a)
    gf, lf = small(make_solver(pkg, dev, g))
    torch.testing.assert_close(la, lf, rtol=0, atol=0)
    torch.testing.assert_close(ga, gf, rtol=0, atol=0)
