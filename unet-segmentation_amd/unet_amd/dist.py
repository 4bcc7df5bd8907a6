"""Data-parallel plumbing: one process per GPU, torch.distributed (backend
"nccl" = RCCL over xGMI on ROCm; "gloo" for CPU tests).

The reference (scripts/train.py) is single-process; north_star adds DP only:
each rank trains on its own shard of HeLaDataset indices (DistributedSampler
semantics) and the gradients are all-reduced after backward.  The MI355X plan's
backward runs in 9 segments whose gradients are contiguous slices of one flat
buffer, so every finished slice is all-reduced while later segments compute.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's environment
    (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT).  Returns
    (rank, world, local_rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    device = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank, world, local, device


class ShardedIndices:
    """DistributedSampler semantics over n dataset indices: an (optionally
    shuffled, per-epoch seeded) permutation padded by wrap-around to a multiple
    of world, then rank r takes every world-th index starting at r."""

    def __init__(self, n, world, rank, shuffle=True, seed=0):
        if not 0 <= rank < world:
            raise ValueError("rank out of range")
        self.n, self.world, self.rank, self.shuffle, self.seed = n, world, rank, shuffle, seed
        self.epoch = 0
        self.per_rank = math.ceil(n / world)

    def set_epoch(self, epoch):
        self.epoch = epoch

    def indices(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g).tolist()
        else:
            order = list(range(self.n))
        total = self.per_rank * self.world
        order = (order * (total // max(len(order), 1) + 1))[:total]
        return order[self.rank:total:self.world]

    def __iter__(self):
        return iter(self.indices())

    def __len__(self):
        return self.per_rank


class GradBucketReducer:
    """All-reduce (SUM) slices of a flat gradient buffer as they become final.

    ``buckets`` is a list of (start, stop) element ranges of ``flat``; call
    ``reduce(b)`` when bucket b is final (asynchronous), ``wait()`` before the
    optimizer.  The optimizer divides by the world size (the fused SGD takes a
    gradient scale), so the buffer holds the SUM afterwards.

    ``comm_dtype=torch.bfloat16`` sends the buckets as bf16 (half the bytes on
    xGMI: 62 instead of 124 MB per step for the U-Net): each bucket is rounded
    into a bf16 shadow, reduced there and widened back into ``flat`` on
    ``wait()``.  Opt-in (Trainer(comm_dtype=torch.bfloat16)): the ranks' values
    are then summed in bf16 by the collective, so the summation error grows with
    the world size; the default keeps fp32 DDP semantics.

    ``ready(b, stream)``, when given, makes the collective's issuing stream wait
    for everything bucket b depends on beyond the current stream (the plan's
    side-stream weight gradients, unet_plan_wait_segment); the collective is
    then issued from that stream, so later work on the current stream (the
    next backward segment) does not wait for it.

    ``force=True`` (tests only) issues the collectives at world size 1 too,
    where they are the identity: the RCCL path (stream-ordered ``Work.wait``,
    the side-stream issue, the bf16 shadow) then runs on a one-GPU box."""

    def __init__(self, flat, buckets, group=None, comm_dtype=None, ready=None, force=False):
        self.flat = flat
        self.force = bool(force)
        self.issued = 0  # collectives issued so far
        self.buckets = list(buckets)
        self.group = group
        self.works = []
        self.ready = ready
        self.stream = None
        comm_dtype = flat.dtype if comm_dtype is None else comm_dtype  # None: the buffer's own dtype
        self.comm_dtype = comm_dtype
        self.shadow = None if comm_dtype == flat.dtype else torch.empty(flat.numel(), dtype=comm_dtype,
                                                                         device=flat.device)
        cover = sorted(self.buckets)
        for (a, b), (c, d) in zip(cover, cover[1:]):
            if b > c:
                raise ValueError("overlapping gradient buckets")

    @property
    def world(self):
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    @property
    def bytes_per_step(self):
        elem = torch.tensor([], dtype=self.comm_dtype).element_size()
        return sum(z - a for a, z in self.buckets) * elem

    def reduce(self, b):
        if self.world == 1 and not self.force:
            return
        a, z = self.buckets[b]
        if self.ready is None or not self.flat.is_cuda:
            self._issue(a, z)
            return
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=self.flat.device)
        cur = torch.cuda.current_stream(self.flat.device)
        self.stream.wait_stream(cur)       # the segment's input-gradient chain and bucket writes
        self.ready(b, self.stream)         # + its side-stream weight gradients
        with torch.cuda.stream(self.stream):
            self._issue(a, z)

    def _issue(self, a, z):
        self.issued += 1
        if self.shadow is None:
            self.works.append((dist.all_reduce(self.flat[a:z], group=self.group, async_op=True), a, z))
            return
        buf = self.shadow[a:z]
        buf.copy_(self.flat[a:z])
        self.works.append((dist.all_reduce(buf, group=self.group, async_op=True), a, z))

    def reduce_all(self):
        for b in range(len(self.buckets)):
            self.reduce(b)

    def wait(self):
        """Make the current stream wait for every issued collective (and widen
        bf16 buckets back into the flat buffer)."""
        for w, a, z in self.works:
            w.wait()
            if self.shadow is not None:
                self.flat[a:z].copy_(self.shadow[a:z])
        if self.stream is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)
        self.works.clear()


def broadcast_buffers(module, src=0, group=None):
    """DDP buffer semantics: every rank takes rank src's BatchNorm running stats."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    for t in module.buffers():
        dist.broadcast(t, src, group=group)
