"""Autograd-free training step for the MI355X UNet (scripts/train.py loop body).

``Trainer.step(x, targets, weights)`` does exactly what scripts/train.py:114-131
does per minibatch -- zero_grad, forward, WeightedCrossEntropyLoss, backward,
SGD(lr, momentum=0.99).step() -- with the same arithmetic as the drop-in
``UNet``/``WeightedCrossEntropyLoss``/``torch.optim.SGD`` trio, but:

* parameters, gradients and momentum live in three flat fp32 buffers (the
  module's parameters are re-homed as views, so ``state_dict`` is unchanged);
* one persistent plan workspace (no per-step allocation);
* the optimizer is one fused kernel over the flat buffer;
* ``precision="bf16"`` runs the convolution GEMMs on bf16 operands with fp32
  accumulation (configs C3/C5); ``"bf16x3"`` runs them fp32-accurate on the
  bf16 matrix cores (operands split into bf16 hi/lo pairs, three products);
  weights, gradients and the optimizer stay fp32 in every mode;
* with a process group, the backward runs in 9 segments and each segment's
  gradient bucket is all-reduced (RCCL over xGMI) while later segments compute:
  the plan leaves each segment's weight gradients running on its side stream
  (UNET_BWD_DEFER_JOIN), the bucket's collective is issued from a stream that
  waits for them, and the side stream is joined once, before the optimizer;
  gradients are summed in fp32 (``comm_dtype=torch.bfloat16`` halves the xGMI
  bytes, opt-in); every step starts from rank 0's BatchNorm running
  statistics (one flat buffer), as DDP does.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .dist import GradBucketReducer
from .plan import N_SEGMENTS, Plan


def _align4(n):
    return (n + 3) // 4 * 4


class FlatParams:
    """Re-home a module's parameters into one flat buffer (16-B aligned slots)."""

    def __init__(self, module: torch.nn.Module):
        params = list(module.parameters())
        dev = params[0].device
        offs, total = [], 0
        for p in params:
            offs.append(total)
            total += _align4(p.numel())
        self.numel = total
        self.offsets = offs
        self.params = params
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.momentum = torch.zeros(total, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, o in zip(params, offs):
                view = self.flat[o:o + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
        self.grad_views = [self.grad[o:o + p.numel()].view_as(p) for p, o in zip(params, offs)]

    def range_for(self, first, count):
        """Flat-buffer element range holding parameters [first, first+count)."""
        a = self.offsets[first]
        b = self.offsets[first + count] if first + count < len(self.offsets) else self.numel
        return a, b


class FlatBuffers:
    """Re-home a module's floating-point buffers (BatchNorm running statistics)
    into one flat buffer, so that DDP's per-step buffer broadcast is a single
    collective instead of one per tensor."""

    def __init__(self, module: torch.nn.Module):
        bufs = [b for b in module.buffers() if b.is_floating_point()]
        total = sum(b.numel() for b in bufs)
        self.flat = torch.zeros(total, dtype=torch.float32, device=bufs[0].device) if bufs else None
        self.bufs = bufs
        o = 0
        with torch.no_grad():
            for b in bufs:
                view = self.flat[o:o + b.numel()].view_as(b)
                view.copy_(b.data)
                b.data = view
                o += b.numel()

    def version(self):
        """A counter that moves whenever torch writes the buffers: through the
        module's buffer tensors (load_state_dict, reset_running_stats, copy_;
        ``b.data = view`` gave each its own version counter) or through the
        flat tensor.  The plan's HIP kernels bump none of them (the running
        statistics update of a forward is not a rewrite)."""
        return (self.flat._version if self.flat is not None else 0) + sum(b._version for b in self.bufs)


class Trainer:
    def __init__(self, model, batch, height, width, lr=1e-4, momentum=0.99, process_group=None,
                 overlap=True, precision="fp32", comm_dtype=None, broadcast_buffers=True, graph=False,
                 force_collectives=False):
        from .modules import UNet
        if not isinstance(model, UNet):
            raise TypeError("Trainer drives the MI355X UNet")
        self.model = model
        self.lr, self.mom = float(lr), float(momentum)
        self.pg = process_group
        self.overlap = overlap
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self.flat = FlatParams(model)
        self.flat_buffers = FlatBuffers(model)
        # DDP default: every step starts from rank 0's BatchNorm running statistics
        # force_collectives (tests only): issue the buffer broadcast and the bucket
        # all-reduces at world size 1 too, where they are the identity
        self.broadcast_buffers = broadcast_buffers and (self.world > 1 or (force_collectives and self.pg is not None))
        dev = self.flat.flat.device
        self.plan = Plan(batch, model.n_channels, height, width, model.n_classes, precision)
        self.ws = torch.empty(self.plan.workspace_bytes, dtype=torch.uint8, device=dev)
        self.state = [t for _, t in model.state_dict(keep_vars=True).items()]
        self.param_tab = _lib.ptr_array(self.state)
        self.grad_tab = _lib.ptr_array(self.flat.grad_views)
        k, oh, ow = model.n_classes, self.plan.out_h, self.plan.out_w
        self.logits = torch.empty((batch, k, oh, ow), dtype=torch.float32, device=dev)
        self.dlogits = torch.empty_like(self.logits)
        self.loss = torch.empty((), dtype=torch.float32, device=dev)
        self.acc = torch.empty(8, dtype=torch.float64, device=dev)
        from .modules import LabelCheck
        self.labels = LabelCheck()
        self._capturing = False
        self.first_step = True
        # segment s+1's input gradients do not wait for segment s's weight
        # gradients (False: join the side stream at every segment end)
        self.defer_join = True
        self.use_graph = bool(graph)
        self._graph = None
        self._graph_key = None
        self._eager_steps = 0
        self.graph_error = None
        # deferred buffer broadcast (round 5): rank 0's running statistics as a
        # forward left them are broadcast into a staging copy beside that step's
        # backward and applied at the next step's start -- DDP's per-step
        # broadcast without a collective ahead of every forward
        self.defer_buffer_bcast = True  # False: the synchronous broadcast ahead of every forward
        self.on_buffers_synced = None   # diagnostics / tests: called with the flat buffers once a step's broadcast landed
        self._bcast_stage = None
        self._bcast_work = None
        self._bcast_version = None
        self._warned_rewrite = False
        self.lib = _lib.load()
        buckets = [self.flat.range_for(*self.plan.segment_grads(s)) for s in range(N_SEGMENTS)]
        # gradient all-reduce dtype: fp32 (DDP semantics) unless the caller asks
        # for bf16 on the wire (half the xGMI bytes; summed in bf16)
        self.comm_dtype = torch.float32 if comm_dtype is None else comm_dtype
        comm_dtype = self.comm_dtype
        self.reducer = GradBucketReducer(self.flat.grad, buckets, process_group, comm_dtype,
                                         ready=lambda b, st: self.plan.wait_segment(b, st), force=force_collectives)
        self.reducer_whole = GradBucketReducer(self.flat.grad, [(0, self.flat.numel)], process_group, comm_dtype,
                                               force=force_collectives)

    @property
    def out_hw(self):
        return self.plan.out_h, self.plan.out_w

    def _check_batch(self, x, targets, weights):
        from .modules import _check_loss_operands
        n, c, h, w = self.plan.shape
        if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()):
            raise RuntimeError("x must be a contiguous float32 HIP tensor")
        if tuple(x.shape) != (n, c, h, w):
            raise ValueError(f"x must be {(n, c, h, w)} (the Trainer's plan shape), got {tuple(x.shape)}")
        if x.device != self.logits.device:
            raise RuntimeError(f"x is on {x.device}, the model on {self.logits.device}")
        _check_loss_operands(self.logits, targets, weights)
        if weights.dtype != torch.float32:
            raise RuntimeError(f"weight_maps must be float32 for the fused loss, got {weights.dtype}")

    def forward_loss(self, x, targets, weights):
        self._check_batch(x, targets, weights)
        if not self._capturing:
            self.labels.check()  # an earlier step's out-of-range target (raises IndexError)
        self.plan.forward(self.param_tab, x, self.logits, self.ws, True)
        n, k, h, w = self.logits.shape
        ts = (ctypes.c_int64 * 3)(*targets.stride())
        wsd = (ctypes.c_int64 * 3)(*weights.stride())
        _lib.check(self.lib.unet_wce_fwd_bwd(self.logits.data_ptr(), targets.data_ptr(), weights.data_ptr(), n, k, h,
                                             w, ts, wsd, self.loss.data_ptr(), self.dlogits.data_ptr(),
                                             ctypes.c_float(1.0), self.acc.data_ptr(), _lib.stream_of(x.device)),
                   "unet_wce_fwd_bwd")
        if not self._capturing:
            self.labels.record(self.acc)
        return self.loss

    def backward_and_reduce(self, x):
        if self.pg is None or not self.overlap:
            self.plan.backward(self.param_tab, self.grad_tab, x, self.dlogits, self.ws, 0, N_SEGMENTS)
            if self.pg is not None:
                self.reducer_whole.reduce_all()
                self.reducer_whole.wait()
            return
        for s in range(N_SEGMENTS):
            # segment s's weight gradients stay on the plan's side stream (no join):
            # segment s+1's input gradients start at once
            self.plan.backward(self.param_tab, self.grad_tab, x, self.dlogits, self.ws, s, s + 1,
                               defer_join=self.defer_join)
            self.reducer.reduce(s)  # bucket s is final once its side-stream work is: all-reduce it meanwhile
        self.plan.join(x.device)
        self.reducer.wait()

    def optimizer_step(self):
        fp = self.flat
        _lib.check(self.lib.unet_sgd_momentum(fp.flat.data_ptr(), fp.grad.data_ptr(), fp.momentum.data_ptr(),
                                              fp.numel, ctypes.c_float(self.lr), ctypes.c_float(self.mom),
                                              ctypes.c_float(1.0 / self.world), int(self.first_step),
                                              _lib.stream_of(fp.flat.device)), "unet_sgd_momentum")
        self.first_step = False

    def step(self, x, targets, weights):
        """One train.py step; returns the (device) loss without synchronising.

        Single-process training with ``graph=True`` replays the whole step
        (forward, loss, backward, SGD: ~190 kernels on two streams) as one
        hipGraph once the GEMM autotuner has settled (from the third step on,
        for the same input tensors); any other call runs eagerly."""
        if (self._graph is not None and not self.plan.timing_on and
                self._graph_key == self._key(x, targets, weights)):
            self.labels.check()  # an earlier step's out-of-range target (raises IndexError)
            self._graph.replay()
            # the replayed loss kernel wrote this step's label flag into acc: queue
            # its host copy behind the replay like an eager step does
            self.labels.record(self.acc)
            return self.loss
        if self._graph is not None and self._graph_key[1:] != (self.lr, self.mom):
            self._graph = None  # stale hyper-parameters: capture again after this eager step
            self._eager_steps = 1
        bufs = self.flat_buffers.flat if self.broadcast_buffers else None
        if bufs is not None:
            self._apply_buffer_broadcast(bufs)
            if self.on_buffers_synced is not None:
                self.on_buffers_synced(bufs)
        loss = self.forward_loss(x, targets, weights)
        if bufs is not None and self.defer_buffer_bcast:
            # the backward and SGD never touch the running statistics: rank 0's
            # post-forward values (what DDP broadcasts at the next forward) travel
            # beside them into the staging copy
            if self._bcast_stage is None:
                self._bcast_stage = torch.empty_like(bufs)
            self._bcast_stage.copy_(bufs)
            self._bcast_work = torch.distributed.broadcast(self._bcast_stage, 0, group=self.pg, async_op=True)
            self._bcast_version = self.flat_buffers.version()
        self.backward_and_reduce(x)
        self.optimizer_step()
        self._eager_steps += 1
        if (self.use_graph and self.pg is None and self._graph is None and self._eager_steps >= 2 and
                not self.plan.timing_on):
            self._capture(x, targets, weights)
        return loss

    def _apply_buffer_broadcast(self, bufs):
        """DDP's start-of-step buffer broadcast: every rank starts the step from
        rank 0's running statistics.  Deferred form: the staged copy of rank 0's
        statistics as its previous forward left them (broadcast beside that
        step's backward).  Rank 0 keeps its own buffers -- they ARE rank 0's
        statistics, and so include any rewrite made since the staging
        (load_state_dict, reset_running_stats) -- every other rank takes the
        staged copy, overwriting anything it changed locally, as DDP does.

        Every rank issues the same collectives whatever happened locally (the
        round-5 fallback broadcast was a rank-local decision and could pair
        mismatched collectives).  The one case the staged copy
        cannot cover is a rewrite on rank 0 after the staging: the other ranks
        then start one step from rank 0's previous values (their batch
        statistics, gradients and weights are unaffected -- BatchNorm trains on
        batch statistics -- and the next step's broadcast brings rank 0's
        rewritten values).  Rank 0 warns once; ``sync_buffers()`` on every rank
        after such a rewrite gives DDP's values at once.  The first step (no
        staged copy) broadcasts synchronously on every rank."""
        work, self._bcast_work = self._bcast_work, None
        if work is None:
            torch.distributed.broadcast(bufs, 0, group=self.pg)
            return
        work.wait()  # NCCL: the current stream waits; gloo: the host does
        if torch.distributed.get_rank(self.pg) != 0:
            bufs.copy_(self._bcast_stage)
        elif self.flat_buffers.version() != self._bcast_version and not self._warned_rewrite:
            self._warned_rewrite = True
            import warnings
            warnings.warn("BatchNorm running statistics were rewritten on rank 0 between Trainer steps: the other "
                          "ranks start this step from the previous broadcast; call Trainer.sync_buffers() on every "
                          "rank after such a change for DDP's values at once", RuntimeWarning, stacklevel=3)

    def check_targets(self):
        """Wait for every step issued so far and raise IndexError if any of them
        met a target outside [0, K) other than ignore_index -100 (torch's
        CrossEntropyLoss raises at once; the fused loss flags it on the device
        and the flag is otherwise read at the next step).  Call it at the end of
        an epoch / run so the last step's labels are checked too."""
        self.labels.check(wait=True)

    def _key(self, x, targets, weights):
        # lr / momentum are baked into the captured SGD launch: a change re-captures
        return (tuple((t.data_ptr(), tuple(t.shape), tuple(t.stride())) for t in (x, targets, weights)),
                self.lr, self.mom)

    def _capture(self, x, targets, weights):
        """Capture one eager-equivalent step (first_step is already False, so
        the captured SGD is the steady-state update).  A capture failure leaves
        the trainer eager."""
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        self._capturing = True
        try:
            with torch.cuda.graph(g):
                self.forward_loss(x, targets, weights)
                self.backward_and_reduce(x)
                self.optimizer_step()
        except Exception as e:  # pragma: no cover - depends on the runtime
            self.use_graph = False
            self.graph_error = repr(e)
            torch.cuda.synchronize()
            return
        finally:
            self._capturing = False
        # (capture launches nothing: the step that triggered it has already run eagerly)
        self._graph, self._graph_key = g, self._key(x, targets, weights)

    def sync_buffers(self, src=0):
        """Broadcast rank-src BatchNorm running statistics now (``step`` does it
        at the start of every step unless ``broadcast_buffers=False``)."""
        if self.pg is None:
            return
        if self._bcast_work is not None:  # a staged broadcast in flight: retire it, a fresh one follows
            self._bcast_work.wait()
            self._bcast_work = None
        if self.flat_buffers.flat is not None:
            torch.distributed.broadcast(self.flat_buffers.flat, src, group=self.pg)
        for name, t in self.model.named_buffers():
            if not t.is_floating_point():
                torch.distributed.broadcast(t, src, group=self.pg)
