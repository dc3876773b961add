"""Data-parallel logic on CPU with the gloo backend, world_size 2:
  * GradBuckets (bucketed, backward-order, overlapped all-reduce over the flat
    gradient arena) averages gradients exactly like one rank on the full batch;
  * rank sharding follows DistributedSampler semantics;
  * validation Dice counts / loss are summed across ranks.
The per-rank gradients come from the CPU oracle (the engine itself needs a GPU;
its bucket callbacks are exercised in the GPU tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import mmseg_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


FEATS = [8, 16, 32, 64, 128]


def _setup():
    torch.manual_seed(0)
    p = O.init_unet3d(2, 3, FEATS)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 2, 32, 32, 32, generator=g)
    y = torch.randint(0, 3, (4, 32, 32, 32), generator=g)
    return p, x, y


def _flat_grads(p, x, y):
    pp = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    O.dice_ce_loss(O.unet3d_forward(pp, x), y).backward()
    return torch.cat([pp[k].grad.reshape(-1) for k in p])


def _worker(rank, world, port, q):
    try:
        _work(rank, world, port, q)
    except Exception as e:  # surface worker failures instead of a queue timeout
        import traceback
        q.put((rank, "error", traceback.format_exc(), None))


def _work(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import mmseg_amd  # noqa: F401
    from mmseg_amd.distributed import ddp
    torch.set_num_threads(2)
    p, x, y = _setup()
    idx = ddp.shard_indices(4, rank, world)
    grad = _flat_grads(p, x[idx], y[idx])
    sizes = [v.numel() for v in p.values()]
    offs = list(np.cumsum([0] + sizes[:-1]))
    gb = ddp.GradBuckets(grad, [int(o) for o in offs], sizes, bucket_mb=0.05)
    assert len(gb.buckets) > 3
    for i in reversed(range(len(sizes))):      # backward order
        gb.param_ready(i)
    gb.finish()
    counts = torch.tensor([float(rank + 1), 2.0 * rank])
    ddp.allreduce_sum_(counts)
    q.put((rank, idx, grad.numpy(), counts.numpy()))
    dist.destroy_process_group()


def test_bucketed_allreduce_equals_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in procs]
    for r in res:
        assert r[1] != "error", r[2]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    res.sort(key=lambda t: t[0])
    assert res[0][1] == [0, 2] and res[1][1] == [1, 3]
    assert np.array_equal(res[0][2], res[1][2]), "ranks disagree after all-reduce"
    p, x, y = _setup()
    full = _flat_grads(p, x, y).numpy()
    err = np.abs(res[0][2] - full).max() / np.abs(full).max()
    assert err < 1e-5, err
    assert np.array_equal(res[0][3], np.array([3.0, 2.0]))


def test_bucket_layout_covers_arena_once():
    import mmseg_amd  # noqa: F401
    from mmseg_amd.distributed.ddp import GradBuckets
    sizes = [1000, 5, 300000, 7, 20000, 1]
    offs = list(np.cumsum([0] + sizes[:-1]))
    gb = GradBuckets(torch.zeros(sum(sizes)), [int(o) for o in offs], sizes, bucket_mb=0.1)
    cover = sorted((lo, hi) for (_, _, lo, hi) in gb.buckets)
    assert cover[0][0] == 0 and cover[-1][1] == sum(sizes)
    assert all(a[1] == b[0] for a, b in zip(cover, cover[1:]))
    assert sorted(i for b in gb.buckets for i in range(b[0], b[1])) == list(range(len(sizes)))


@pytest.mark.parametrize("n,w", [(4, 2), (5, 2), (32, 6), (2, 4), (7, 8), (1, 3)])
def test_shard_indices_match_distributed_sampler(n, w):
    """Every rank gets ceil(n/W) samples (wrap-around padding), exactly DistributedSampler(shuffle=False)'s
    order, so no rank runs an extra train_step and hangs the others in the gradient all-reduce."""
    import mmseg_amd  # noqa: F401
    from mmseg_amd.distributed.ddp import shard_indices
    from torch.utils.data.distributed import DistributedSampler
    shards = [shard_indices(n, r, w) for r in range(w)]
    assert len({len(s) for s in shards}) == 1 and len(shards[0]) == -(-n // w)
    for r in range(w):
        assert shards[r] == list(DistributedSampler(range(n), num_replicas=w, rank=r, shuffle=False))
