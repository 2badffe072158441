"""Round-5 cases on the HIP path (needs an MI355X):

  * the path-chunked phase pipeline on the column-split kernels (16-row
    workgroups) at a batch whose row count is not a multiple of the 64-row
    padding (M = 96, N = 50: R = 4896, Rp = 4928): the last chunk runs the
    padding tiles, so a context that ran a larger batch before gives the
    fresh one-chunk step bit for bit (no stale loss partial or weight-gradient
    row of the earlier batch is summed);
  * the streams ordered by value write / wait or by events give the same
    training steps;
  * a prefetch held back for the two-stream step changes no result;
  * the chain weight gradients piped per path chunk (HJB shape) give the
    one-chunk step bit for bit."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_pkg

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


def _model(pkg, dev, g, env):
    layers = [int(v) for v in g["layers"]]
    D = layers[0] - 1
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = pkg.BlackScholesBarenblatt(g["Xi"], 1.0, 1024, 50, D, layers, "NAIS-Net", "Sine", device=dev)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    m.params.copy_(torch.from_numpy(g["params"]).to(dev))
    return m


def _step(m, M, seed):
    loss = torch.empty(1, device=m.params.device)
    m.solver.loss_grad(m.params, M, 50, m._device_xi(0, M), seed=seed, grad=m.grad, loss=loss)
    torch.cuda.synchronize()
    return loss.cpu().clone(), m.grad.cpu().clone()


def test_chunked_column_split_step_with_row_padding(pkg, dev):
    g = _load("g2_north_star.npz")
    chunked = _model(pkg, dev, g, {"DBSDE_CS": "1", "DBSDE_CHUNKS": "2"})
    fresh = _model(pkg, dev, g, {"DBSDE_CS": "1", "DBSDE_CHUNKS": "1"})
    _step(chunked, 1024, seed=3)          # fills every row buffer past the small batch's rows
    l2, g2 = _step(chunked, 96, seed=5)   # R = 4896, Rp = 4928: padding tiles in the last chunk
    l1, g1 = _step(fresh, 96, seed=5)
    assert torch.isfinite(l1).all() and float(l1) > 0.0
    torch.testing.assert_close(l2, l1, rtol=0, atol=0)
    torch.testing.assert_close(g2, g1, rtol=0, atol=0)


def test_stream_order_by_events_matches_value_ops(pkg, dev):
    """The chunk fork / join and the prefetch order as stream value write /
    wait (default) or as events (DBSDE_STREAM_ORDER=events, the fallback under
    kernel serialisation and counter collection): four prefetched training
    steps end on the same parameters bit for bit."""
    g = _load("g2_north_star.npz")
    runs = []
    for env in ({}, {"DBSDE_STREAM_ORDER": "events"}):
        m = _model(pkg, dev, g, env)
        opt = m.new_optimizer_state("Adam", 1e-3)
        for it in range(4):
            m.device_step(opt, 1e-3, seed=11 + it, next_seed=12 + it)
        torch.cuda.synchronize()
        runs.append(m.params.detach().cpu().clone())
    assert torch.isfinite(runs[0]).all()
    torch.testing.assert_close(runs[0], runs[1], rtol=0, atol=0)


def test_held_back_prefetch_on_the_second_stream_is_the_same_step(pkg, dev):
    """At the north-star shape the step runs the two-stream pipeline, so a
    prefetched batch is held back and rolled out on the step's second stream
    after its weight-gradient slices (engine.hip launch_deferred_on): four
    device steps with the next batch prefetched end on the same parameters
    bit for bit as four without prefetching; a prefetch that no step consumes
    (a different seed) leaves the steps unchanged as well."""
    g = _load("g2_north_star.npz")
    runs = []
    for mode in ("none", "next", "stale"):
        m = _model(pkg, dev, g, {})
        opt = m.new_optimizer_state("Adam", 1e-3)
        for it in range(4):
            nxt = {"none": None, "next": 22 + it, "stale": 1000 + it}[mode]
            m.device_step(opt, 1e-3, seed=21 + it, next_seed=nxt)
        torch.cuda.synchronize()
        runs.append(m.params.detach().cpu().clone())
    assert torch.isfinite(runs[0]).all()
    torch.testing.assert_close(runs[1], runs[0], rtol=0, atol=0)
    torch.testing.assert_close(runs[2], runs[0], rtol=0, atol=0)


def test_chain_weight_gradients_piped_per_chunk(pkg, dev):
    """Config 4's shape (HJB, FC-Sine [101,256x4,1], M = 2048, N = 20) runs
    the two-chunk pipeline, and its split-bf16 chain weight gradients are
    launched per chunk (row splits of chunk 0 after its phase C, the rest
    after chunk 1's): the step is bit for bit the one-chunk step whose
    weight gradients run after the phase section."""
    D, M, N = 100, 2048, 20
    layers = [D + 1] + 4 * [256] + [1]
    rs = np.random.RandomState(41)
    params = None
    Xi = torch.zeros(D, device=dev)
    res = []
    for chunks in ("2", "1"):
        old = os.environ.get("DBSDE_CHUNKS")
        os.environ["DBSDE_CHUNKS"] = chunks
        try:
            s = pkg.NativeSolver("FC", layers, "Sine", pkg.ProblemSpec(sig_b=float(np.sqrt(2.0)), phi_zz=1.0, g="log"),
                                 1.0, dev)
        finally:
            if old is None:
                os.environ.pop("DBSDE_CHUNKS", None)
            else:
                os.environ["DBSDE_CHUNKS"] = old
        if params is None:
            params = torch.from_numpy(rs.normal(scale=0.05, size=s.nparams).astype(np.float32)).to(dev)
        grad, loss = torch.empty_like(params), torch.empty(1, device=dev)
        s.loss_grad(params, M, N, Xi, seed=9, grad=grad, loss=loss)
        torch.cuda.synchronize()
        res.append((float(loss), grad.cpu().clone()))
    assert np.isfinite(res[0][0])
    assert res[0][0] == res[1][0]
    torch.testing.assert_close(res[0][1], res[1][1], rtol=0, atol=0)
