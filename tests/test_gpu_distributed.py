"""Two ranks (gloo, both on cuda:0) running the native step must reproduce the
single-process step over the same global batch:
  * throughput mode: device Philox increments keyed by the GLOBAL path index,
    [grad|loss] all-reduce, replicated Adam (what bench.py times);
  * parity mode: the reference's train() loop, every rank drawing the global
    numpy batch and uploading only its slice of paths.
Needs a GPU.  RCCL (the "nccl" backend) needs one device per rank, so on a
one-GPU box it runs as a single rank: the process group comes up over RCCL,
the [grad | loss] buffer goes through an RCCL all-reduce, and the steps equal
the non-distributed ones bit for bit.  Two-rank runs use gloo."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, load_pkg

pytestmark = pytest.mark.gpu
D, M, N = 8, 64, 10
LAYERS = [D + 1, 16, 16, 16, 16, 1]


def _model(world, rank):
    pkg = load_pkg()
    torch.manual_seed(0)
    Xi = np.array([1.0, 0.5] * (D // 2))[None, :]
    m = pkg.BlackScholesBarenblatt(Xi, 1.0, M, N, D, LAYERS, "NAIS-Net", "Sine", device=torch.device("cuda:0"))
    m.rank, m.world = rank, world
    return m


def _steps(m, k=3):
    opt = m.new_optimizer_state()
    losses = []
    for it in range(k):
        losses.append(float(m.device_step(opt, 1e-3, seed=it)))
    torch.cuda.synchronize()
    return m.params.cpu().numpy(), losses


def _train(m, k=3):
    np.random.seed(5)
    m.train(k, 1e-3)
    torch.cuda.synchronize()
    return m.params.cpu().numpy(), list(m.training_loss)


def _worker(rank, world, port, q, what):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if what == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model(world, rank)
        if what == "nccl":
            p, l = _steps(m)
            # the step's all-reduce on its device buffer, through RCCL
            buf = m._gradbuf.clone()
            dist.all_reduce(m._gradbuf)
            torch.cuda.synchronize()
            q.put((rank, p, l, bool(torch.equal(buf, m._gradbuf)), dist.get_backend()))
        else:
            q.put((rank,) + (_steps(m) if what == "steps" else _train(m)))
    finally:
        dist.destroy_process_group()


def _two_ranks(what, world=2):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, what)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_two_ranks_train_parity_mode_matches_one_process():
    res = _two_ranks("train")
    p1, l1 = _train(_model(1, 0))
    (_, pa, la), (_, pb, lb) = res
    np.testing.assert_array_equal(pa, pb)
    np.testing.assert_allclose(la, l1, rtol=1e-5)
    np.testing.assert_allclose(pa, p1, rtol=0, atol=2e-6)


def test_two_ranks_match_one_process():
    res = _two_ranks("steps")
    p1, l1 = _steps(_model(1, 0))
    (_, pa, la), (_, pb, lb) = res
    np.testing.assert_array_equal(pa, pb)                       # replicas identical
    np.testing.assert_allclose(la, l1, rtol=1e-5)               # global loss = sum of shard losses
    np.testing.assert_allclose(pa, p1, rtol=0, atol=2e-6)       # Adam steps agree


def test_rccl_backend_single_rank():
    """RCCL on the box: a one-rank "nccl" process group, the native steps, and
    an RCCL all-reduce of the step's [grad | loss] device buffer (identity at
    one rank); the steps equal the non-distributed ones bit for bit."""
    ((_, p, l, same, backend),) = _two_ranks("nccl", world=1)
    p1, l1 = _steps(_model(1, 0))
    assert backend == "nccl" and same
    np.testing.assert_array_equal(p, p1)
    np.testing.assert_array_equal(l, l1)
