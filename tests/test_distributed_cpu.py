"""World-size-2 data parallelism on CPU (gloo): the FBSNN host path shards the
minibatch's paths over ranks, all-reduces [grad | loss] once per step and runs
the optimizer replicated.  The native solver is replaced by an oracle-backed
stand-in (test infrastructure), so this checks the sharding / reduction logic
exactly as bench.py and train() drive it, without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT, load_pkg
from oracle import timeparallel as tp

CASE = os.path.join(GOLDEN, "g1_deep_bsb_NAIS-Net_Sine.npz")


class OracleSolver:
    """Same call surface as NativeSolver, computed by oracle/timeparallel.py."""

    def __init__(self, mode, layers, act, problem):
        self.mode, self.layers, self.act, self.problem = mode, layers, act, problem
        self.nb = layers[0] - 1

    def loss_grad(self, params, M, N, Xi, t=None, W=None, grad=None, loss=None, X=None, Y=None, Z=None, **kw):
        D = self.layers[0] - 1
        out = tp.loss_grad(params.double().numpy(), self.mode, self.layers, self.act, self.problem,
                           t.double().numpy().reshape(M, N + 1), W.double().numpy().reshape(M, N + 1, D),
                           Xi.double().numpy().reshape(-1, D))
        if grad is not None:
            grad.copy_(torch.from_numpy(out["grad"]).float())
        loss.copy_(torch.tensor([out["loss"]], dtype=torch.float32))
        if X is not None:
            X.copy_(torch.from_numpy(out["X"]).float())
        if Y is not None:
            Y.copy_(torch.from_numpy(out["Y"]).float())

    def optimizer_step(self, params, grad, m, v, kind, lr, max_norm, step, **kw):
        assert kind == "Adam"
        m.lerp_(grad, 0.1)
        v.mul_(0.999).addcmul_(grad, grad, value=0.001)
        denom = (v.sqrt() / np.sqrt(1 - 0.999 ** step)).add_(1e-8)
        params.addcdiv_(m, denom, value=-lr / (1 - 0.9 ** step))


def make_model(world, rank):
    pkg = load_pkg()
    g = np.load(CASE)
    layers = [int(v) for v in g["layers"]]
    obj = object.__new__(pkg.BlackScholesBarenblatt)
    obj.device = torch.device("cpu")
    obj.D, obj.M, obj.N, obj.T = layers[0] - 1, int(g["M"]), int(g["N"]), float(g["T"])
    obj.layers, obj.Mm, obj._L = layers, None, None
    obj.spec = pkg.ProblemSpec(sig_a=0.4, phi_r=0.05, phi_c=1.0, g="sumsq")
    obj.training_loss, obj.iteration = [], []
    obj.Xi = torch.from_numpy(g["Xi"]).float()
    obj.params = torch.from_numpy(g["params"]).clone()
    obj._gradbuf = torch.zeros(obj.params.numel() + 1)
    obj.grad = obj._gradbuf[:-1]
    obj.solver = OracleSolver(str(g["mode"]), layers, str(g["activation"]), "bsb")
    obj.rank, obj.world = rank, world
    return obj, torch.from_numpy(g["t"]), torch.from_numpy(g["W"])


def run_steps(obj, t, W, steps=2):
    opt = obj.new_optimizer_state()
    losses = []
    for _ in range(steps):
        loss, _ = obj.train_step(t, W, opt, "Adam", 1e-3)
        losses.append(float(loss))
    return obj.params.clone().numpy(), losses


def run_train(obj, iters=3, seed=11):
    """The reference train() loop (host numpy stream, each rank uploads its slice)."""
    np.random.seed(seed)
    obj.train(iters, 1e-3)
    return obj.params.clone().numpy(), list(obj.training_loss)


def _worker(rank, world, port, q, what):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obj, t, W = make_model(world, rank)
        q.put((rank,) + (run_steps(obj, t, W) if what == "steps" else run_train(obj)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _two_ranks(what):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, what)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_two_rank_train_equals_single_process():
    """train() with the reference's numpy stream: every rank draws the global
    batch and uploads its slice; two ranks == one process (parity mode)."""
    res = _two_ranks("train")
    single, _, _ = make_model(1, 0)
    p1, l1 = run_train(single)
    (_, pa, la), (_, pb, lb) = res
    np.testing.assert_array_equal(pa, pb)
    np.testing.assert_allclose(la, l1, rtol=1e-6)
    np.testing.assert_allclose(pa, p1, rtol=0, atol=1e-6)


def test_two_rank_data_parallel_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, "steps")) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single, t, W = make_model(1, 0)
    p1, l1 = run_steps(single, t, W)
    (_, pa, la), (_, pb, lb) = res
    np.testing.assert_array_equal(pa, pb)                  # replicas stay identical
    np.testing.assert_allclose(la, l1, rtol=1e-6)          # summed loss == full-batch loss
    np.testing.assert_allclose(pa, p1, rtol=0, atol=1e-6)  # same update as one process


def test_indivisible_batch_is_rejected():
    obj, t, W = make_model(3, 0)
    with pytest.raises(ValueError):
        obj._local_slice(8)


def test_q3_problems_refuse_sharding():
    """the D == 1 squeeze broadcast sums over all paths; a sharded
    rank cannot reproduce it, so the split is refused."""
    pkg = load_pkg()
    obj, t, W = make_model(2, 0)
    obj.layers = [2, 16, 16, 16, 16, 1]
    obj.spec = pkg.ProblemSpec(mu_a=0.01, sig_a=0.25, phi_r=0.01, g="call_sum", strike=1.0, q3=True)
    with pytest.raises(ValueError, match="q3"):
        obj._local_slice(8)
