"""Op-by-op forwards of the reference submodules on the per-op C-ABI.

The drop-in ``UNet.forward`` runs the whole network as one HIP plan.  The
reference's submodules are callable on their own as well --
``DoubleConv.forward`` (models/unet_model.py:20-21), ``Down.forward`` (:32-33),
``Up.forward(x1, x2_cropped)`` (:50-54), ``OutConv.forward`` (:62-63) -- and
the reference's autograd differentiates an eval-mode forward too.  Both go
through this module: every op is a HIP kernel of libunet_hip.so behind its own
``torch.autograd.Function`` (fp32 GEMMs):

* 3x3 valid conv: the first conv (any Ci -> 64, from the NCHW input) by the
  direct kernels of the plan's stage 1 (``unet_conv_first_*``), the others by
  the implicit-GEMM entry points (``unet_conv3x3_{fwd,dgrad,wgrad}``);
* BatchNorm2d + ReLU (``unet_bn_relu_{fwd,bwd}``; train: batch statistics and
  the running-statistics update, eval: the running statistics as constants);
* MaxPool2d(2) (``unet_maxpool2_*``), ConvTranspose2d(2, 2)
  (``unet_convT2_*``), the 1x1 head (``unet_conv1x1_*``).

Activations between the ops are channels_last tensors (NHWC in memory, the
layout the kernels read); the center crop is a view and the skip concat a
``torch.cat`` copy, as in the reference.  There is no PyTorch fallback: a CPU
tensor raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading

import torch

from . import _lib

_CL = torch.channels_last


def _lib_and_stream(t):
    if not t.is_cuda:
        raise RuntimeError("the MI355X UNet blocks have no CPU path: move the tensors to the HIP device")
    if t.dtype != torch.float32:
        raise RuntimeError(f"the MI355X UNet blocks compute in float32, got {t.dtype}")
    return _lib.load(), _lib.stream_of(t.device)


# GEMM precision of the block ops.  Inside torch.autocast("cuda", bfloat16) the
# reference's convs run on bf16 operands with fp32 accumulation (and return
# bf16); the blocks then run their conv / convT GEMMs the same way
# (op_precision UNET_PREC_BF16: operands rounded to bf16 at staging, fp32
# accumulation), in the backward too (its ops inherit the forward's precision,
# as autocast's bf16 saved tensors make the reference's backward bf16).
# op_precision is process-wide in the library: it is set around each call
# under a lock and put back to fp32.
_PREC_LOCK = threading.Lock()
_PREC_BF16 = 1  # UNET_PREC_BF16 (include/unet_hip.h)


def _autocast_bf16():
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


@contextlib.contextmanager
def _gemm_precision(lib, bf16):
    if not bf16:
        yield
        return
    with _PREC_LOCK:
        _lib.check(lib.unet_set_tuning(b"op_precision", _PREC_BF16), "unet_set_tuning")
        try:
            yield
        finally:
            lib.unet_set_tuning(b"op_precision", 0)


def _block_in(x):
    """A block's input as the kernels read it: float32 (a bf16 / fp16 tensor
    from an autocast region is widened -- exact -- outside the autograd
    Functions, so its gradient comes back in its own dtype)."""
    if x.is_floating_point() and x.dtype != torch.float32 and _autocast_bf16():
        return x.float()
    return x


def _block_out(y):
    """Under bf16 autocast the reference's blocks return bf16 (their last op is a
    conv, or a BatchNorm / ReLU of one, on bf16 operands)."""
    return y.to(torch.bfloat16) if _autocast_bf16() else y


def _cl(t):
    return t.contiguous(memory_format=_CL)


def _nhwc(n, c, h, w, like):
    return torch.empty((n, c, h, w), dtype=torch.float32, device=like.device, memory_format=_CL)


def _ws(nbytes, like):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=like.device)


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class _FirstConv(torch.autograd.Function):
    """The first conv (models/unet_model.py:11 with in_channels = n_channels):
    any Ci -> 64 from an NCHW input."""

    @staticmethod
    def forward(ctx, x, w, b):
        lib, st = _lib_and_stream(x)
        x = x.contiguous()
        n, ci, h, wd = x.shape
        y = _nhwc(n, 64, h - 2, wd - 2, x)
        _lib.check(lib.unet_conv_first_fwd(_p(x), n, ci, h, wd, _p(w.contiguous()), _p(b.contiguous()), _p(y), st),
                   "unet_conv_first_fwd")
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        lib, st = _lib_and_stream(dy)
        dy = _cl(dy)
        n, ci, h, wd = x.shape
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w)
        db = torch.empty(64, dtype=torch.float32, device=x.device)
        ws = _ws(lib.unet_conv_first_ws_bytes(n, ci, h, wd), x)
        _lib.check(lib.unet_conv_first_bwd(_p(x), _p(dy), n, ci, h, wd, _p(w.contiguous()), _p(dx), _p(dw), _p(db),
                                           _p(ws), st), "unet_conv_first_bwd")
        return dx, dw, db


class _Conv3x3(torch.autograd.Function):
    """nn.Conv2d(k=3, padding=0) (models/unet_model.py:11, 15) as implicit GEMM."""

    @staticmethod
    def forward(ctx, x, w, b, bf16=False):
        lib, st = _lib_and_stream(x)
        x = _cl(x)
        n, ci, h, wd = x.shape
        co = w.shape[0]
        y = _nhwc(n, co, h - 2, wd - 2, x)
        ws = _ws(lib.unet_conv_ws_bytes(n, h, wd, ci, co), x)
        with _gemm_precision(lib, bf16):
            _lib.check(lib.unet_conv3x3_fwd(_p(x), n, h, wd, ci, _p(w.contiguous()), _p(b.contiguous()), co, None,
                                            None, _p(y), _p(ws), st), "unet_conv3x3_fwd")
        ctx.save_for_backward(x, w)
        ctx.bf16 = bf16
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        lib, st = _lib_and_stream(dy)
        dy = _cl(dy)
        n, ci, h, wd = x.shape
        co = w.shape[0]
        ws = _ws(lib.unet_conv_ws_bytes(n, h, wd, ci, co), x)
        dx = None
        with _gemm_precision(lib, ctx.bf16):
            if ctx.needs_input_grad[0]:
                dx = _nhwc(n, ci, h, wd, x)
                _lib.check(lib.unet_conv3x3_dgrad(_p(dy), n, h, wd, ci, _p(w.contiguous()), co, _p(dx), _p(ws), st),
                           "unet_conv3x3_dgrad")
            dw = torch.empty_like(w)
            db = torch.empty(co, dtype=torch.float32, device=x.device)
            _lib.check(lib.unet_conv3x3_wgrad(_p(x), _p(dy), n, h, wd, ci, co, _p(dw), _p(db), _p(ws), st),
                       "unet_conv3x3_wgrad")
        return dx, dw, db, None


class _BNReLU(torch.autograd.Function):
    """nn.BatchNorm2d followed by nn.ReLU (models/unet_model.py:12-13, 16-17)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, nbt, training, momentum, eps):
        lib, st = _lib_and_stream(x)
        x = _cl(x)
        n, c, h, w = x.shape
        y = _nhwc(n, c, h, w, x)
        mean = torch.empty(c, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        ws = _ws(lib.unet_bn_relu_ws_bytes(n, h, w, c), x)
        _lib.check(lib.unet_bn_relu_fwd(_p(x), n, h, w, c, _p(gamma), _p(beta), _p(rm), _p(rv),
                                        _p(nbt) if training else None, ctypes.c_float(momentum),
                                        ctypes.c_float(eps), int(training), 1, _p(y), _p(mean), _p(invstd), _p(ws),
                                        st), "unet_bn_relu_fwd")
        ctx.training = bool(training)
        ctx.save_for_backward(x, y, gamma, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, mean, invstd = ctx.saved_tensors
        lib, st = _lib_and_stream(dy)
        dy = _cl(dy)
        n, c, h, w = x.shape
        dx = _nhwc(n, c, h, w, x)
        dgamma = torch.empty_like(gamma)
        dbeta = torch.empty_like(gamma)
        ws = _ws(lib.unet_bn_relu_ws_bytes(n, h, w, c), x)
        _lib.check(lib.unet_bn_relu_bwd(_p(x), _p(y), _p(dy), n, h, w, c, _p(gamma), _p(mean), _p(invstd),
                                        int(ctx.training), 1, _p(dx), _p(dgamma), _p(dbeta), _p(ws), st),
                   "unet_bn_relu_bwd")
        return dx, dgamma, dbeta, None, None, None, None, None, None


class _MaxPool2(torch.autograd.Function):
    """nn.MaxPool2d(2) (models/unet_model.py:28): floor mode, the first max of a
    window (row-major) takes the gradient."""

    @staticmethod
    def forward(ctx, x):
        lib, st = _lib_and_stream(x)
        x = _cl(x)
        n, c, h, w = x.shape
        y = _nhwc(n, c, h // 2, w // 2, x)
        arg = torch.empty((n, h // 2, w // 2, c), dtype=torch.uint8, device=x.device)
        _lib.check(lib.unet_maxpool2_fwd(_p(x), n, h, w, c, _p(y), _p(arg), st), "unet_maxpool2_fwd")
        ctx.save_for_backward(arg)
        ctx.shape = (n, c, h, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        lib, st = _lib_and_stream(dy)
        dy = _cl(dy)
        n, c, h, w = ctx.shape
        dx = _nhwc(n, c, h, w, dy).zero_()  # the floor-dropped last row / column get no gradient
        _lib.check(lib.unet_maxpool2_bwd(_p(dy), _p(arg), n, h, w, c, _p(dx), st), "unet_maxpool2_bwd")
        return dx


class _ConvT2(torch.autograd.Function):
    """nn.ConvTranspose2d(k=2, s=2) (models/unet_model.py:45)."""

    @staticmethod
    def forward(ctx, x, w, b, bf16=False):
        lib, st = _lib_and_stream(x)
        x = _cl(x)
        n, ci, h, wd = x.shape
        co = w.shape[1]
        y = _nhwc(n, co, 2 * h, 2 * wd, x)
        ws = _ws(lib.unet_conv_ws_bytes(n, h, wd, ci, co), x)
        with _gemm_precision(lib, bf16):
            _lib.check(lib.unet_convT2_fwd(_p(x), n, h, wd, ci, _p(w.contiguous()), _p(b.contiguous()), co, _p(y),
                                           _p(ws), st), "unet_convT2_fwd")
        ctx.save_for_backward(x, w)
        ctx.bf16 = bf16
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        lib, st = _lib_and_stream(dy)
        dy = _cl(dy)
        n, ci, h, wd = x.shape
        co = w.shape[1]
        dx = _nhwc(n, ci, h, wd, x)
        dw = torch.empty_like(w)
        db = torch.empty(co, dtype=torch.float32, device=x.device)
        ws = _ws(lib.unet_conv_ws_bytes(n, h, wd, ci, co), x)
        with _gemm_precision(lib, ctx.bf16):
            _lib.check(lib.unet_convT2_bwd(_p(x), _p(dy), n, h, wd, ci, _p(w.contiguous()), co, _p(dx), _p(dw),
                                           _p(db), _p(ws), st), "unet_convT2_bwd")
        return dx, dw, db, None


class _Conv1x1(torch.autograd.Function):
    """OutConv's nn.Conv2d(64, n_classes, 1) (models/unet_model.py:59); logits NCHW."""

    @staticmethod
    def forward(ctx, x, w, b):
        lib, st = _lib_and_stream(x)
        x = _cl(x)
        n, c, h, wd = x.shape
        k = w.shape[0]
        out = torch.empty((n, k, h, wd), dtype=torch.float32, device=x.device)
        _lib.check(lib.unet_conv1x1_fwd(_p(x), n, h, wd, c, _p(w.contiguous()), _p(b.contiguous()), k, _p(out), st),
                   "unet_conv1x1_fwd")
        ctx.save_for_backward(x, w)
        return out

    @staticmethod
    def backward(ctx, dl):
        x, w = ctx.saved_tensors
        lib, st = _lib_and_stream(dl)
        dl = dl.contiguous()
        n, c, h, wd = x.shape
        k = w.shape[0]
        dx = _nhwc(n, c, h, wd, x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w)
        db = torch.empty(k, dtype=torch.float32, device=x.device)
        ws = _ws(lib.unet_conv1x1_ws_bytes(k), x)
        _lib.check(lib.unet_conv1x1_bwd(_p(x), _p(dl), n, h, wd, c, _p(w.contiguous()), k, _p(dx), _p(dw), _p(db),
                                        _p(ws), st), "unet_conv1x1_bwd")
        return dx, dw, db


def conv3x3(conv, x):
    """nn.Conv2d(k=3, padding=0) on the HIP kernels: the first conv of the
    network (Ci not a multiple of 64, 64 outputs) by the direct stage-1 kernels,
    the others by implicit GEMM."""
    ci, co = conv.in_channels, conv.out_channels
    if ci % 64:
        if co != 64:
            raise ValueError(f"3x3 conv {ci}->{co}: the MI355X blocks take Ci % 64 != 0 only for the first conv "
                             "(64 outputs)")
        return _FirstConv.apply(x, conv.weight, conv.bias)
    if co % 64:
        raise ValueError(f"3x3 conv {ci}->{co}: output channels must be a multiple of 64")
    return _Conv3x3.apply(x, conv.weight, conv.bias, _autocast_bf16())


def bn_relu(bn, x):
    """nn.BatchNorm2d + nn.ReLU with the module's mode, momentum and eps."""
    if bn.momentum is None or not bn.track_running_stats or not bn.affine:
        raise NotImplementedError("the MI355X BatchNorm block takes the reference's BatchNorm2d(C) "
                                  "(affine, tracked running statistics, momentum 0.1)")
    return _BNReLU.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                         bn.training, float(bn.momentum), float(bn.eps))


def _double_conv(m, x):
    seq = m.double_conv
    return bn_relu(seq[4], conv3x3(seq[3], bn_relu(seq[1], conv3x3(seq[0], x))))


def _up_conv(m, x):
    return _ConvT2.apply(x, m.up.weight, m.up.bias, _autocast_bf16())


def double_conv(m, x):
    """DoubleConv.forward (models/unet_model.py:20-21)."""
    return _block_out(_double_conv(m, _block_in(x)))


def down(m, x):
    """Down.forward (models/unet_model.py:32-33): MaxPool2d(2) then DoubleConv."""
    return _block_out(_double_conv(m.maxpool_conv[1], _MaxPool2.apply(_block_in(x))))


def up_conv(m, x):
    """The Up block's ConvTranspose2d(k=2, s=2) (models/unet_model.py:45, 51)."""
    return _block_out(_up_conv(m, _block_in(x)))


def up(m, x1, x2_cropped):
    """Up.forward (models/unet_model.py:50-54): upsample x1, concatenate
    [x2_cropped, x1] along channels (skip first), DoubleConv."""
    x1 = _up_conv(m, _block_in(x1))
    return _block_out(_double_conv(m.conv, torch.cat([_cl(_block_in(x2_cropped)), x1], dim=1)))


def out_conv(m, x):
    """OutConv.forward (models/unet_model.py:62-63)."""
    return _block_out(_Conv1x1.apply(_block_in(x), m.conv.weight, m.conv.bias))


def unet_forward(model, x):
    """UNet.forward (models/unet_model.py:105-146) op by op on these blocks."""
    x1 = _double_conv(model.inc, _block_in(x))
    x2 = _double_conv(model.down1.maxpool_conv[1], _MaxPool2.apply(x1))
    x3 = _double_conv(model.down2.maxpool_conv[1], _MaxPool2.apply(x2))
    x4 = _double_conv(model.down3.maxpool_conv[1], _MaxPool2.apply(x3))
    x5 = _double_conv(model.down4.maxpool_conv[1], _MaxPool2.apply(x4))
    x = x5
    for blk, skip in ((model.up1, x4), (model.up2, x3), (model.up3, x2), (model.up4, x1)):
        x_up = _up_conv(blk, x)
        crop = model._center_crop(skip, x_up.size()[2:])
        x = _double_conv(blk.conv, torch.cat([_cl(crop), x_up], dim=1))
    # fp32 logits, as the plan's UNet.forward returns them in every precision
    return _Conv1x1.apply(x, model.outc.conv.weight, model.outc.conv.bias)
