"""Round-6 cases on the HIP path (needs an MI355X): the prefetch ordering.

  * a prefetched batch no step consumes ("stale": prefetch seed X, run seed Y,
    repeat) must never be rolled out into the path buffer the running step
    reads (engine.hip launch_deferred_on falls back to pf_stream avoiding that
    buffer): the X / Y / Z exports, loss and gradient of every step equal a
    context without prefetching, bit for bit, at the north-star shape (two
    path chunks, so the held-back rollout runs on the second stream);
  * consecutive steps on alternating streams with no ordering by the caller
    (dbsde_set_stream follows torch's current stream): the context orders the
    new stream after the old one on every switch, and a prefetched rollout
    joined into one stream is waited for by a consumer on another
    (engine.hip wait_pending), so the steps equal the single-stream,
    unprefetched ones bit for bit."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_pkg

pytestmark = pytest.mark.gpu
M, N = 1024, 50


@pytest.fixture(scope="module")
def pkg():
    return load_pkg()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def g():
    z = np.load(os.path.join(GOLDEN, "g2_north_star.npz"))
    return {k: z[k] for k in z.files}


def _model(pkg, dev, g):
    layers = [int(v) for v in g["layers"]]
    m = pkg.BlackScholesBarenblatt(g["Xi"], 1.0, M, N, layers[0] - 1, layers, "NAIS-Net", "Sine", device=dev)
    m.params.copy_(torch.from_numpy(g["params"]).to(dev))
    return m


def _outs(m):
    D = m.state_dim
    return dict(loss=torch.empty(1, device=m.device), X=torch.empty(M * (N + 1) * D, device=m.device),
                Y=torch.empty(M * (N + 1), device=m.device), Z=torch.empty(M * (N + 1) * D, device=m.device),
                grad=torch.empty_like(m.params))


def _run_steps(m, seeds, prefetch, streams=None):
    xi = m._device_xi(0, M)
    torch.cuda.synchronize()     # params / xi written on the default stream
    res = []
    for i, seed in enumerate(seeds):
        st = streams[i % len(streams)] if streams else torch.cuda.current_stream(m.device)
        with torch.cuda.stream(st):
            if prefetch is not None and prefetch(i) is not None:
                m.solver.prefetch(M, N, xi, seed=prefetch(i))
            o = _outs(m)
            m.solver.loss_grad(m.params, M, N, xi, seed=seed, grad=o["grad"], loss=o["loss"], X=o["X"], Y=o["Y"],
                               Z=o["Z"])
        res.append(o)            # no synchronisation between steps: the ordering is what is tested
    torch.cuda.synchronize()
    return [{k: v.cpu().clone() for k, v in o.items()} for o in res]


def _same(a, b):
    for ra, rb in zip(a, b):
        for k in ra:
            torch.testing.assert_close(ra[k], rb[k], rtol=0, atol=0, msg=k)


def test_stale_prefetch_never_overwrites_the_running_step(pkg, dev, g):
    seeds = [31, 32, 33, 34, 35]
    base = _run_steps(_model(pkg, dev, g), seeds, None)
    assert all(torch.isfinite(r["loss"]).all() for r in base)
    stale = _run_steps(_model(pkg, dev, g), seeds, lambda i: 5000 + i)
    _same(stale, base)
    # a mix: the next batch, then a stale one, then the next again
    mixed = _run_steps(_model(pkg, dev, g), seeds, lambda i: (seeds[i + 1] if i + 1 < len(seeds) else None)
                       if i % 2 == 0 else 7000 + i)
    _same(mixed, base)


def test_prefetch_consumed_on_another_stream(pkg, dev, g):
    seeds = [41, 42, 43, 44, 45, 46]
    base = _run_steps(_model(pkg, dev, g), seeds, None)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    swapped = _run_steps(_model(pkg, dev, g), seeds, lambda i: seeds[i + 1] if i + 1 < len(seeds) else None,
                         streams=[s1, s2])
    _same(swapped, base)


@pytest.mark.parametrize("Mr,Nr,D", [(1024, 50, 100), (37, 13, 100), (5, 3, 7)])
def test_two_pass_rollout_equals_single_pass(pkg, dev, monkeypatch, Mr, Nr, D):
    """The in-step device rollout in two passes (rollout_draw_kernel +
    rollout_chain_kernel, paths.hpp) against rollout4_kernel
    (DBSDE_ROLLOUT2=0, read at context creation): X, Y, Z, loss and gradient
    bit for bit, also at ragged M and at N not a multiple of the 4-step Philox
    block or the 8-step load-ahead."""
    layers = [D + 1, 16, 16, 16, 16, 1]
    xi = np.random.RandomState(3).uniform(0.5, 1.5, (1, D)).astype(np.float32)

    def run(flag):
        if flag is None:
            monkeypatch.delenv("DBSDE_ROLLOUT2", raising=False)
        else:
            monkeypatch.setenv("DBSDE_ROLLOUT2", flag)
        torch.manual_seed(4)
        m = pkg.BlackScholesBarenblatt(xi, 1.0, Mr, Nr, D, layers, "NAIS-Net", "Sine", device=dev)
        o = dict(loss=torch.empty(1, device=dev), X=torch.empty(Mr * (Nr + 1) * D, device=dev),
                 Y=torch.empty(Mr * (Nr + 1), device=dev), Z=torch.empty(Mr * (Nr + 1) * D, device=dev),
                 grad=torch.empty_like(m.params))
        m.solver.loss_grad(m.params, Mr, Nr, m._device_xi(0, Mr), seed=77, grad=o["grad"], loss=o["loss"], X=o["X"],
                           Y=o["Y"], Z=o["Z"])
        torch.cuda.synchronize()
        return {k: v.cpu() for k, v in o.items()}

    two, one = run(None), run("0")
    assert torch.isfinite(two["X"]).all()
    for k in two:
        torch.testing.assert_close(two[k], one[k], rtol=0, atol=0, msg=k)


def test_large_batch_is_the_sum_of_its_halves(pkg, dev, g):
    """M = 16384 paths per GPU (16x the north star: R = 835,584 rows, 13,056
    phase workgroups per launch, the two-chunk pipeline with prefetch-free
    in-step rollouts) against its two halves, drawn with the device Philox
    keyed by the global path index (path0 = 0 and 8192): X bit for bit, the
    loss and the gradient as sums over the paths (DeepBSDE.py:231-241)."""
    Ml, Nl = 16384, 50
    m = _model(pkg, dev, g)
    D = m.state_dim
    xi = m._device_xi(0, M)

    def run(M, path0):
        o = dict(loss=torch.empty(1, device=dev), X=torch.empty(M * (Nl + 1) * D, device=dev),
                 Y=torch.empty(M * (Nl + 1), device=dev), grad=torch.empty_like(m.params))
        m.solver.loss_grad(m.params, M, Nl, xi, seed=99, path0=path0, grad=o["grad"], loss=o["loss"], X=o["X"],
                           Y=o["Y"])
        torch.cuda.synchronize()
        return {k: v.cpu().double() for k, v in o.items()}

    full = run(Ml, 0)
    a, b = run(Ml // 2, 0), run(Ml // 2, Ml // 2)
    assert torch.isfinite(full["loss"]).all() and torch.isfinite(full["grad"]).all()
    torch.testing.assert_close(full["X"], torch.cat([a["X"], b["X"]]), rtol=0, atol=0)
    torch.testing.assert_close(full["Y"], torch.cat([a["Y"], b["Y"]]), rtol=0, atol=1e-5 * float(full["Y"].abs().max()))
    assert float(full["loss"]) == pytest.approx(float(a["loss"] + b["loss"]), rel=1e-5)
    g2 = a["grad"] + b["grad"]
    torch.testing.assert_close(full["grad"], g2, rtol=0, atol=2e-5 * float(g2.abs().max()))
