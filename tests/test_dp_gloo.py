"""Data-parallel plumbing on CPU with the gloo backend (world size 2).

The MI355X trainer all-reduces the 9 backward-segment buckets of one flat
gradient buffer (unet_amd.dist.GradBucketReducer) and the fused SGD divides by
the world size.  Here every rank computes its shard's gradients with the CPU
oracle, lays them out exactly like unet_amd.train.FlatParams, runs the real
reducer over the plan's segment buckets, and applies SGD(momentum 0.99) with
scale 1/world.  The DP parity oracle of SURVEY.md §8e: the result must equal
the host-side average of the two shards' gradients (per-replica BatchNorm
statistics, the DDP default), and both ranks must end with identical weights.
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from oracle import unet_oracle as O
from oracle import fixtures as F


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _layout(shapes):
    offs, total = [], 0
    for shp in shapes:
        offs.append(total)
        total += (int(np.prod(shp)) + 3) // 4 * 4
    return offs, total


def _shard_grads(rank, h=188):
    params = O.hash_init(1, 2, seed=21, bn_random=True)
    x, t, w = F.make_inputs(100 + rank, 1, 1, h)
    net = O.UNetOracle(params)
    logits, cache, _ = net.forward(x)
    _, dl = O.weighted_ce(logits, t, w)
    return params, net.backward(dl, cache)


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        from unet_amd.dist import GradBucketReducer
        from unet_amd.plan import Plan, N_SEGMENTS
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        torch.set_num_threads(2)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        params, grads = _shard_grads(rank)
        names = [k for k in O.param_shapes(1, 2) if not O.is_buffer(k)]
        offs, total = _layout([params[k].shape for k in names])
        flat = torch.zeros(total, dtype=torch.float64)
        for k, o in zip(names, offs):
            flat[o:o + grads[k].size] = torch.from_numpy(np.asarray(grads[k], np.float64).ravel())
        plan = Plan(1, 1, 188, 188, 2)  # host-only: segment table
        buckets = []
        for s in range(N_SEGMENTS):
            f, k = plan.segment_grads(s)
            a = offs[f]
            b = offs[f + k] if f + k < len(offs) else total
            buckets.append((a, b))
        red = GradBucketReducer(flat, buckets)
        for s in range(N_SEGMENTS):
            red.reduce(s)
        red.wait()
        # fused SGD semantics: p -= lr * (momentum buffer of g / world); first step buf = g
        lr = 1e-4
        newp = {}
        for k, o in zip(names, offs):
            g = flat[o:o + grads[k].size].numpy().reshape(params[k].shape) / world
            newp[k], _ = O.sgd_momentum_step(np.asarray(params[k], np.float64), g, None, lr=lr)
        q.put((rank, {k: newp[k] for k in names}, None))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(600)
def test_dp_allreduce_matches_shard_average():
    ctx = mp.get_context("spawn")  # fork would inherit the parent's OpenMP/BLAS pools (deadlock)
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, newp, err = q.get(timeout=580)
        assert err is None, err
        out[rank] = newp
    for p in procs:
        p.join(timeout=60)
    # host-side DP oracle: average the two shards' gradients
    p0, g0 = _shard_grads(0)
    _, g1 = _shard_grads(1)
    for k, v in out[0].items():
        ref, _ = O.sgd_momentum_step(np.asarray(p0[k], np.float64), (g0[k] + g1[k]) / 2, None, lr=1e-4)
        np.testing.assert_allclose(v, ref, rtol=0, atol=1e-12, err_msg=k)
        np.testing.assert_array_equal(out[1][k], v)


def test_sharded_indices_cover_dataset():
    from unet_amd.dist import ShardedIndices
    n = 76  # scripts/train.py:82-84: 84 frames, 10 % validation -> 76 training samples
    for world in (1, 2, 3, 8):
        shards = [ShardedIndices(n, world, r, shuffle=True, seed=3) for r in range(world)]
        for s in shards:
            s.set_epoch(5)
        idx = [i for s in shards for i in s.indices()]
        assert len(idx) == world * shards[0].per_rank
        assert set(idx) == set(range(n))
        assert all(len(s.indices()) == len(s) for s in shards)
        if world * shards[0].per_rank == n:
            assert len(set(idx)) == n  # disjoint when n divides evenly


def _bf16_worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        from unet_amd.dist import GradBucketReducer
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = torch.Generator().manual_seed(7 + rank)
        flat = torch.randn(1000, generator=g, dtype=torch.float32)
        red = GradBucketReducer(flat, [(0, 400), (400, 1000)], comm_dtype=torch.bfloat16)
        assert red.bytes_per_step == 2000
        red.reduce(1)
        red.reduce(0)
        red.wait()
        q.put((rank, flat.numpy().copy(), None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(300)
def test_bf16_bucket_allreduce():
    """comm_dtype=bf16 (opt-in): each bucket goes over the wire
    as bf16 and comes back widened; equals the bf16 sum of the bf16-rounded
    shards, identical on both ranks."""
    import torch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bf16_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, v, err = q.get(timeout=280)
        assert err is None, err
        out[rank] = v
    for p in procs:
        p.join(timeout=60)
    shards = [torch.randn(1000, generator=torch.Generator().manual_seed(7 + r), dtype=torch.float32) for r in range(2)]
    ref = (shards[0].bfloat16() + shards[1].bfloat16()).float().numpy()
    np.testing.assert_array_equal(out[0], out[1])
    np.testing.assert_array_equal(out[0], ref)


def test_flat_buffers_rehome_running_stats():
    """Trainer's FlatBuffers: every floating BatchNorm buffer becomes a view of
    one flat tensor (one broadcast per step), values and state_dict unchanged."""
    import torch
    from unet_amd.train import FlatBuffers
    m = torch.nn.Sequential(torch.nn.Conv2d(1, 4, 3), torch.nn.BatchNorm2d(4), torch.nn.BatchNorm2d(4))
    with torch.no_grad():
        for b in m.buffers():
            if b.is_floating_point():
                b.copy_(torch.rand_like(b))
    before = {k: v.clone() for k, v in m.state_dict().items()}
    fb = FlatBuffers(m)
    assert fb.flat.numel() == 4 * 4
    after = m.state_dict()
    for k, v in before.items():
        assert torch.equal(after[k], v), k
    fb.flat.fill_(3.0)
    assert all(torch.all(b == 3.0) for b in m.buffers() if b.is_floating_point())
    assert all(b.dtype == torch.int64 for b in m.buffers() if not b.is_floating_point())
