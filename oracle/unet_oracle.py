"""CPU oracle for the U-Net training / inference hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``unet-segmentation_amd/``)
imports this module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker (or as the timed CPU
baseline).  The HIP path never falls back to it.

This is a NumPy restatement (float64 by default) of the reference algorithm
SaurabhIndi/unet-segmentation @ 2025-07-25.  Every function cites the reference
file:line it restates (paths relative to the reference root):

* models/unet_model.py  -- UNet / DoubleConv / Down / Up / OutConv / _center_crop
* utils/losses.py       -- WeightedCrossEntropyLoss
* scripts/train.py      -- center_crop_tensor, init_weights, SGD(momentum=0.99)
* scripts/predict.py    -- eval forward + softmax[:,1] > 0.5 mask
* scripts/predict1.py   -- overlap-tile margin (in - out = 184 per axis)
* utils/metrics.py      -- calculate_iou

The arithmetic inside those files is PyTorch's (torch.nn.Conv2d, BatchNorm2d,
MaxPool2d, ConvTranspose2d, CrossEntropyLoss, optim.SGD); it is restated here
from the published semantics of those ops.

Parity pinning: ``tests/golden/make_golden.py`` imports the reference modules in
the build container (torch 2.10 CPU, float64) and writes the fixtures under
``tests/golden/``; ``tests/test_oracle_golden.py`` checks this oracle against
them.  So the oracle is pinned to the reference itself, not only to the
restatement.

Layout: activations are NHWC internally (that is the layout the HIP path uses
too); parameters use PyTorch's shapes (Conv2d OIHW, ConvTranspose2d IOHW) so
they map 1:1 onto the reference ``state_dict`` keys.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

BN_EPS = 1e-5          # nn.BatchNorm2d default (models/unet_model.py:12,16)
BN_MOMENTUM = 0.1      # nn.BatchNorm2d default

# (name, in_channels, out_channels) of every DoubleConv, in state_dict order.
# models/unet_model.py:73-82
_ENCODER = [("inc", None, 64), ("down1", 64, 128), ("down2", 128, 256),
            ("down3", 256, 512), ("down4", 512, 1024)]
_DECODER = [("up1", 1024, 512), ("up2", 512, 256), ("up3", 256, 128), ("up4", 128, 64)]


def _dc_prefix(block: str) -> str:
    """state_dict prefix of a block's DoubleConv (models/unet_model.py:9, 27-29, 46)."""
    if block == "inc":
        return "inc.double_conv."
    if block.startswith("down"):
        return f"{block}.maxpool_conv.1.double_conv."
    return f"{block}.conv.double_conv."


def param_shapes(n_channels: int = 1, n_classes: int = 2) -> "OrderedDict[str, tuple]":
    """Parameter + buffer schema of ``UNet(n_channels, n_classes)`` in state_dict order.

    models/unet_model.py:66-85 (bilinear=False -> ConvTranspose2d, :45).
    """
    s: "OrderedDict[str, tuple]" = OrderedDict()

    def dc(prefix, cin, cout):
        s[prefix + "0.weight"] = (cout, cin, 3, 3)
        s[prefix + "0.bias"] = (cout,)
        for k in ("1",):
            s[prefix + k + ".weight"] = (cout,)
            s[prefix + k + ".bias"] = (cout,)
            s[prefix + k + ".running_mean"] = (cout,)
            s[prefix + k + ".running_var"] = (cout,)
            s[prefix + k + ".num_batches_tracked"] = ()
        s[prefix + "3.weight"] = (cout, cout, 3, 3)
        s[prefix + "3.bias"] = (cout,)
        s[prefix + "4.weight"] = (cout,)
        s[prefix + "4.bias"] = (cout,)
        s[prefix + "4.running_mean"] = (cout,)
        s[prefix + "4.running_var"] = (cout,)
        s[prefix + "4.num_batches_tracked"] = ()

    for name, cin, cout in _ENCODER:
        dc(_dc_prefix(name), n_channels if cin is None else cin, cout)
    for name, cin, cout in _DECODER:
        s[f"{name}.up.weight"] = (cin, cin // 2, 2, 2)
        s[f"{name}.up.bias"] = (cin // 2,)
        dc(_dc_prefix(name), cin // 2 + cout, cout)
    s["outc.conv.weight"] = (n_classes, 64, 1, 1)
    s["outc.conv.bias"] = (n_classes,)
    return s


def bn_cancelled(name: str) -> bool:
    """Biases whose gradient is analytically zero in train mode: every conv bias
    inside a DoubleConv (a BatchNorm follows) and every ConvTranspose2d bias (its
    output only feeds a conv that feeds a BatchNorm).  SURVEY.md §7 'Hard parts'."""
    return name.endswith(("double_conv.0.bias", "double_conv.3.bias", ".up.bias"))


def is_bn_param(name: str) -> bool:
    """BatchNorm2d affine parameters (weight / bias of double_conv.1 and .4)."""
    return name.endswith(("double_conv.1.weight", "double_conv.1.bias", "double_conv.4.weight",
                          "double_conv.4.bias"))


def is_buffer(name: str) -> bool:
    return name.endswith(("running_mean", "running_var", "num_batches_tracked"))


# ----------------------------------------------------------------------------
# Deterministic counter-based generator (build-defined).
# splitmix64(seed, tensor index, element index) -> uniform (0,1) -> Box-Muller.
# ----------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash_uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """n float64 uniforms in (0,1) from counter (seed, stream, i)."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0x100000001B3 + stream * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF)
        z = _splitmix64(np.arange(n, dtype=np.uint64) + base * np.uint64(0x632BE59BD9B4E019))
    return ((z >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def hash_normal(seed: int, stream: int, n: int) -> np.ndarray:
    u1 = hash_uniform(seed, 2 * stream, n)
    u2 = hash_uniform(seed, 2 * stream + 1, n)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def hash_init(n_channels: int = 1, n_classes: int = 2, seed: int = 0,
              bn_random: bool = False) -> "OrderedDict[str, np.ndarray]":
    """Build-defined deterministic stand-in for ``model.apply(init_weights)``.

    scripts/train.py:54-61: Conv2d weights ~ kaiming_normal(fan_out, relu) =
    N(0, 2/(Co*kh*kw)), conv bias 0, BN gamma 1 / beta 0.  ConvTranspose2d is NOT
    an nn.Conv2d, so it keeps PyTorch's default init: kaiming_uniform(a=sqrt(5))
    = U(-1/sqrt(fan_in), 1/sqrt(fan_in)) with fan_in = weight.size(1)*2*2, same
    bound for its bias.  Values come from the counter hash so the GPU tests can
    regenerate them without committing 124 MB of weights.

    ``bn_random``/non-zero biases are used by parity tests so that every
    parameter has a visible effect (zero biases hide bias-path bugs).
    """
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for i, (name, shape) in enumerate(param_shapes(n_channels, n_classes).items()):
        n = int(np.prod(shape)) if shape else 1
        if name.endswith("num_batches_tracked"):
            out[name] = np.zeros((), np.int64)
            continue
        if name.endswith("running_mean"):
            out[name] = np.zeros(shape, np.float32)
            continue
        if name.endswith("running_var"):
            out[name] = np.ones(shape, np.float32)
            continue
        if name.endswith(".up.weight") or name.endswith(".up.bias"):
            wshape = shape if name.endswith("weight") else None
            co = (wshape[1] if wshape else shape[0])
            fan_in = co * 4
            bound = 1.0 / np.sqrt(fan_in)
            v = (2.0 * hash_uniform(seed, i, n) - 1.0) * bound
            out[name] = v.reshape(shape).astype(np.float32)
            continue
        if len(shape) == 4:  # Conv2d weight
            fan_out = shape[0] * shape[2] * shape[3]
            v = hash_normal(seed, i, n) * np.sqrt(2.0 / fan_out)
            out[name] = v.reshape(shape).astype(np.float32)
            continue
        # 1-D: conv bias, BN weight, BN bias
        is_bn_w = name.split(".")[-2] in ("1", "4") and name.endswith("weight")
        is_bn_b = name.split(".")[-2] in ("1", "4") and name.endswith("bias")
        if bn_random:
            u = hash_uniform(seed, i, n)
            if is_bn_w:
                v = 0.5 + u            # gamma in (0.5, 1.5)
            elif is_bn_b:
                v = 0.2 * (u - 0.5)
            else:
                v = 0.1 * (u - 0.5)    # conv / head bias
        else:
            v = np.ones(n) if is_bn_w else np.zeros(n)
        out[name] = v.reshape(shape).astype(np.float32)
    return out


# ----------------------------------------------------------------------------
# bf16 operand rounding (the HIP path's UNET_PREC_BF16 GEMMs).
# ----------------------------------------------------------------------------
def round_bf16(a):
    """Round to the nearest bf16 (ties to even), as gfx950's v_cvt_pk_bf16_f32
    and torch's float32 -> bfloat16 cast do; the value is taken as float32
    first (the HIP path rounds fp32 activations).  Returns float64 values."""
    f = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    u = f.view(np.uint32).astype(np.uint64)
    u = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) & np.uint64(0xFFFF0000)
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


# ----------------------------------------------------------------------------
# Primitive ops (NHWC activations).
# ----------------------------------------------------------------------------
def conv_valid_fwd(x, w, b):
    """nn.Conv2d(k, padding=0) forward (models/unet_model.py:11,15; 1x1 head :60).

    x (N,H,W,Ci), w (Co,Ci,kh,kw), b (Co,) -> (N,H-kh+1,W-kw+1,Co).
    """
    N, H, W, Ci = x.shape
    Co, _, kh, kw = w.shape
    Ho, Wo = H - kh + 1, W - kw + 1
    out = np.empty((N * Ho * Wo, Co), dtype=x.dtype)
    out[:] = b.astype(x.dtype)
    for ky in range(kh):
        for kx in range(kw):
            xt = np.ascontiguousarray(x[:, ky:ky + Ho, kx:kx + Wo, :]).reshape(-1, Ci)
            out += xt @ w[:, :, ky, kx].astype(x.dtype).T
    return out.reshape(N, Ho, Wo, Co)


def conv_valid_bwd(x, w, dy, need_dx=True):
    """Autograd of conv_valid_fwd: (dx, dw, db).  dx is the full correlation of dy
    with the flipped kernel; dw sums x ⊗ dy over all output pixels."""
    N, H, W, Ci = x.shape
    Co, _, kh, kw = w.shape
    Ho, Wo = H - kh + 1, W - kw + 1
    dyf = dy.reshape(-1, Co)
    db = dyf.sum(0)
    dw = np.empty(w.shape, dtype=dy.dtype)
    dx = np.zeros_like(x, dtype=dy.dtype) if need_dx else None
    for ky in range(kh):
        for kx in range(kw):
            xt = np.ascontiguousarray(x[:, ky:ky + Ho, kx:kx + Wo, :]).reshape(-1, Ci)
            dw[:, :, ky, kx] = dyf.T @ xt
            if need_dx:
                dx[:, ky:ky + Ho, kx:kx + Wo, :] += (dyf @ w[:, :, ky, kx].astype(dy.dtype)).reshape(N, Ho, Wo, Ci)
    return dx, dw, db


def bn_train_fwd(x, gamma, beta, eps=BN_EPS):
    """nn.BatchNorm2d training forward (models/unet_model.py:12,16): batch mean,
    biased variance over (N,H,W).  Returns y, (xhat, invstd), mean, unbiased var."""
    C = x.shape[-1]
    xf = x.reshape(-1, C)
    M = xf.shape[0]
    mean = xf.mean(0)
    var = ((xf - mean) ** 2).mean(0)
    invstd = 1.0 / np.sqrt(var + eps)
    xhat = (xf - mean) * invstd
    y = xhat * gamma + beta
    var_unb = var * M / max(M - 1, 1)
    return y.reshape(x.shape), (xhat.reshape(x.shape), invstd), mean, var_unb


def bn_update_running(rm, rv, mean, var_unb, momentum=BN_MOMENTUM):
    """running_mean/var update with momentum 0.1 and the unbiased variance."""
    return (1 - momentum) * rm + momentum * mean, (1 - momentum) * rv + momentum * var_unb


def bn_eval_fwd(x, gamma, beta, rm, rv, eps=BN_EPS):
    """nn.BatchNorm2d eval forward (scripts/predict.py:70 model.eval())."""
    return (x - rm) / np.sqrt(rv + eps) * gamma + beta


def bn_train_bwd(dy, cache, gamma):
    xhat, invstd = cache
    C = dy.shape[-1]
    dyf = dy.reshape(-1, C)
    xh = xhat.reshape(-1, C)
    M = dyf.shape[0]
    dbeta = dyf.sum(0)
    dgamma = (dyf * xh).sum(0)
    dx = (gamma * invstd / M) * (M * dyf - dbeta - xh * dgamma)
    return dx.reshape(dy.shape), dgamma, dbeta


def relu_fwd(x):
    """nn.ReLU(inplace=True) (models/unet_model.py:13,17)."""
    return np.maximum(x, 0)


def relu_bwd(dy, y):
    """threshold_backward: gradient passes where the OUTPUT is > 0."""
    return dy * (y > 0)


def maxpool2_fwd(x):
    """nn.MaxPool2d(2) (models/unet_model.py:28): 2x2 stride 2, floor mode.

    Returns (y, argmax) with argmax in 0..3 = row-major index inside the window;
    on ties the FIRST maximum wins (strict '>' scan, SURVEY.md §7 'tie rule')."""
    N, H, W, C = x.shape
    Ho, Wo = H // 2, W // 2
    xc = x[:, :2 * Ho, :2 * Wo, :]
    win = np.stack([xc[:, 0::2, 0::2], xc[:, 0::2, 1::2], xc[:, 1::2, 0::2], xc[:, 1::2, 1::2]], axis=0)
    best = win[0].copy()
    arg = np.zeros(best.shape, np.uint8)
    for k in range(1, 4):
        upd = win[k] > best
        best = np.where(upd, win[k], best)
        arg[upd] = k
    return best, arg


def maxpool2_bwd(dy, arg, in_shape):
    N, H, W, C = in_shape
    dx = np.zeros(in_shape, dtype=dy.dtype)
    Ho, Wo = dy.shape[1], dy.shape[2]
    for k in range(4):
        a, b = divmod(k, 2)
        dx[:, a:2 * Ho:2, b:2 * Wo:2, :] += np.where(arg == k, dy, 0)
    return dx


def convT2_fwd(x, w, b):
    """nn.ConvTranspose2d(Ci, Ci//2, kernel_size=2, stride=2) (models/unet_model.py:45).

    x (N,H,W,Ci), w (Ci,Co,2,2), b (Co,) -> (N,2H,2W,Co); non-overlapping taps."""
    N, H, W, Ci = x.shape
    Co = w.shape[1]
    y = np.empty((N, 2 * H, 2 * W, Co), dtype=x.dtype)
    xf = x.reshape(-1, Ci)
    for a in range(2):
        for c in range(2):
            y[:, a::2, c::2, :] = (xf @ w[:, :, a, c].astype(x.dtype)).reshape(N, H, W, Co) + b
    return y


def convT2_bwd(x, w, dy):
    N, H, W, Ci = x.shape
    Co = w.shape[1]
    xf = x.reshape(-1, Ci)
    dx = np.zeros((N * H * W, Ci), dtype=dy.dtype)
    dw = np.empty(w.shape, dtype=dy.dtype)
    for a in range(2):
        for c in range(2):
            d = np.ascontiguousarray(dy[:, a::2, c::2, :]).reshape(-1, Co)
            dx += d @ w[:, :, a, c].astype(dy.dtype).T
            dw[:, :, a, c] = xf.T @ d
    return dx.reshape(x.shape), dw, dy.reshape(-1, Co).sum(0)


def crop_offsets(h, w, th, tw):
    """UNet._center_crop (models/unet_model.py:88-102) / center_crop_tensor
    (scripts/train.py:39-51): start = max(0, (size - target)//2)."""
    return max(0, (h - th) // 2), max(0, (w - tw) // 2)


def center_crop_nhwc(x, th, tw):
    oy, ox = crop_offsets(x.shape[1], x.shape[2], th, tw)
    return x[:, oy:oy + th, ox:ox + tw, :]


def weighted_ce(logits_nchw, target, wmap):
    """WeightedCrossEntropyLoss (utils/losses.py:29-57):
    mean_{n,h,w}( w * (logsumexp_c(l) - l[target]) ).

    Returns (loss, dlogits) with dlogits = w*(softmax - onehot)/(N*H*W)."""
    l = logits_nchw.astype(np.float64)
    m = l.max(1, keepdims=True)
    e = np.exp(l - m)
    s = e.sum(1, keepdims=True)
    lse = (m + np.log(s))[:, 0]
    t = target.astype(np.int64)
    lt = np.take_along_axis(l, t[:, None], 1)[:, 0]
    wmap = np.asarray(wmap, dtype=np.float64)
    pix = (lse - lt) * wmap
    count = pix.size
    loss = pix.sum() / count
    p = e / s
    onehot = np.zeros_like(p)
    np.put_along_axis(onehot, t[:, None], 1.0, 1)
    dlog = (p - onehot) * (wmap[:, None] / count)
    return loss, dlog


def unweighted_ce(logits_nchw, target):
    """nn.CrossEntropyLoss() mean reduction (scripts/train.py:143 validation)."""
    return weighted_ce(logits_nchw, target, np.ones(target.shape))[0]


def sgd_momentum_step(p, g, buf, lr=1e-4, momentum=0.99):
    """torch.optim.SGD(lr, momentum) step (scripts/train.py:97,131):
    buf = g (first step) else momentum*buf + g; p -= lr*buf (dampening 0, no WD)."""
    buf = g.copy() if buf is None else momentum * buf + g
    return p - lr * buf, buf


def calculate_iou(pred, gt):
    """utils/metrics.py:6-37: binarise pred>0, gt>0; |∩|/|∪|; union 0 -> 1.0."""
    p = np.asarray(pred) > 0
    g = np.asarray(gt) > 0
    union = np.logical_or(p, g).sum()
    if union == 0:
        return 1.0
    return float(np.logical_and(p, g).sum() / union)


def center_crop_target(t, th, tw):
    """scripts/train.py:39-51 on an (N,1,H,W) tensor followed by squeeze(1)."""
    oy, ox = crop_offsets(t.shape[-2], t.shape[-1], th, tw)
    return t[:, 0, oy:oy + th, ox:ox + tw]


# ----------------------------------------------------------------------------
# Whole network.
# ----------------------------------------------------------------------------
def output_size(h: int) -> int:
    """Spatial output size of the valid U-Net (models/unet_model.py:151-204):
    512 -> 324, 572 -> 388, 188 -> 4.  Raises for sizes whose down path hits < 1."""
    s = h - 4
    sizes = [s]
    for _ in range(4):
        s = s // 2 - 4
        if s < 1:
            raise ValueError(f"input {h} too small for 4 valid down stages")
        sizes.append(s)
    u = sizes[-1]
    for k in range(4):
        u = 2 * u
        if sizes[3 - k] < u:
            raise ValueError(f"input {h}: skip {sizes[3 - k]} smaller than upsampled {u}")
        u = u - 4
        if u < 1:
            raise ValueError(f"input {h} too small")
    return u


class UNetOracle:
    """Restatement of UNet.forward (models/unet_model.py:105-146) with an explicit
    backward.  ``params`` maps reference state_dict names -> arrays (PyTorch
    shapes); activations are NHWC in ``dtype``.

    ``gemm="bf16"`` restates the HIP path's bf16 arithmetic (UNET_PREC_BF16, the
    reference's convs under torch.autocast(bfloat16)): every 3x3 conv after the
    first, every ConvTranspose2d and their input / weight gradients see both
    operands rounded to bf16 (after the producer's BatchNorm+ReLU), products
    accumulated exactly; every raw conv output (the first conv's too) is
    rounded to bf16 before BatchNorm, as the bf16 plan stores it.  The
    activation gradients the bf16 plan stores between kernels are rounded too:
    every BN-input gradient (after the ReLU mask, before the BN backward and its
    statistics), the pooled-map gradient and the skip gradient.  The first
    conv's arithmetic (Ci <= 4), the 1x1 head, BatchNorm statistics, pooling,
    biases, parameter gradients and the loss stay unrounded."""

    def __init__(self, params, dtype=np.float64, bn_momentum=BN_MOMENTUM, gemm="fp32"):
        if gemm not in ("fp32", "bf16"):
            raise ValueError(gemm)
        self.p = OrderedDict((k, np.asarray(v)) for k, v in params.items())
        self.dtype = dtype
        self.bn_momentum = bn_momentum
        self.gemm = gemm

    def _q(self, a, on=True):
        """GEMM operand as the HIP path sees it."""
        return round_bf16(a).astype(self.dtype) if (on and self.gemm == "bf16") else a

    def _conv_bwd(self, a_in, w, d, need_dx, quant):
        if not (quant and self.gemm == "bf16"):
            return conv_valid_bwd(a_in, w, d, need_dx=need_dx)
        dx, dw, _ = conv_valid_bwd(self._q(a_in), self._q(w), self._q(d), need_dx=need_dx)
        return dx, dw, d.reshape(-1, d.shape[-1]).sum(0)

    def _w(self, name):
        return self.p[name].astype(self.dtype)

    # -- DoubleConv (models/unet_model.py:5-21) --------------------------------
    def _double_conv_fwd(self, pre, x, train, cache, new_buffers):
        d = self.dtype
        outs = []
        a = x
        for conv_i, bn_i in (("0", "1"), ("3", "4")):
            q = not (pre == _dc_prefix("inc") and conv_i == "0")  # first conv: direct fp32 kernel
            y = conv_valid_fwd(self._q(a, q), self._q(self._w(pre + conv_i + ".weight"), q),
                               self._w(pre + conv_i + ".bias"))
            y = self._q(y)  # bf16 plans store every raw conv output in bf16 (BatchNorm sees the rounded values)
            g, b = self._w(pre + bn_i + ".weight"), self._w(pre + bn_i + ".bias")
            if train:
                z, bn_cache, mean, var_unb = bn_train_fwd(y, g, b)
                rm, rv = bn_update_running(self.p[pre + bn_i + ".running_mean"].astype(np.float64),
                                           self.p[pre + bn_i + ".running_var"].astype(np.float64),
                                           mean, var_unb, self.bn_momentum)
                new_buffers[pre + bn_i + ".running_mean"] = rm
                new_buffers[pre + bn_i + ".running_var"] = rv
                new_buffers[pre + bn_i + ".num_batches_tracked"] = self.p[pre + bn_i + ".num_batches_tracked"] + 1
            else:
                z = bn_eval_fwd(y, g, b, self._w(pre + bn_i + ".running_mean"), self._w(pre + bn_i + ".running_var"))
                bn_cache = None
            r = relu_fwd(z).astype(d)
            outs.append((a, bn_cache, r))
            a = r
        cache[pre] = outs
        return a

    def _double_conv_bwd(self, pre, dout, cache, grads, need_dx=True):
        outs = cache[pre]
        d = dout
        for (conv_i, bn_i), (a_in, bn_cache, r) in zip((("3", "4"), ("0", "1")), reversed(outs)):
            d = self._q(relu_bwd(d, r))  # bf16 plans store dz bf16
            d, dg, dbt = bn_train_bwd(d, bn_cache, self._w(pre + bn_i + ".weight"))
            grads[pre + bn_i + ".weight"] = dg
            grads[pre + bn_i + ".bias"] = dbt
            nd = need_dx or conv_i == "3"
            q = not (pre == _dc_prefix("inc") and conv_i == "0")
            d, dw, db = self._conv_bwd(a_in, self._w(pre + conv_i + ".weight"), d, nd, q)
            grads[pre + conv_i + ".weight"] = dw
            grads[pre + conv_i + ".bias"] = db
        return d

    def forward(self, x_nchw, train=True):
        """Returns (logits NCHW, cache, new_buffers)."""
        x = np.ascontiguousarray(np.transpose(np.asarray(x_nchw, dtype=self.dtype), (0, 2, 3, 1)))
        cache, nb = {}, OrderedDict()
        skips = []
        a = self._double_conv_fwd(_dc_prefix("inc"), x, train, cache, nb)
        skips.append(a)
        for k in range(1, 5):
            pooled, arg = maxpool2_fwd(a)
            cache[f"pool{k}"] = (arg, a.shape)
            a = self._double_conv_fwd(_dc_prefix(f"down{k}"), pooled, train, cache, nb)
            if k < 4:
                skips.append(a)
        for k in range(1, 5):
            name = f"up{k}"
            cache[name + ".in"] = a
            up = convT2_fwd(self._q(a), self._q(self._w(name + ".up.weight")), self._w(name + ".up.bias"))
            skip = skips[4 - k]
            cs = center_crop_nhwc(skip, up.shape[1], up.shape[2])
            cache[name + ".crop"] = (skip.shape, crop_offsets(skip.shape[1], skip.shape[2], up.shape[1], up.shape[2]),
                                     cs.shape[-1])
            cat = np.concatenate([cs, up], axis=-1)     # skip first, then upsampled (:131)
            a = self._double_conv_fwd(_dc_prefix(name), cat, train, cache, nb)
        cache["outc.in"] = a
        logits = conv_valid_fwd(a, self._w("outc.conv.weight"), self._w("outc.conv.bias"))
        return np.transpose(logits, (0, 3, 1, 2)), cache, nb

    def backward(self, dlogits_nchw, cache, input_grad=False):
        """Gradients for every parameter (same keys as the reference's named_parameters);
        input_grad: also the gradient of the network input, NCHW (the reference's
        x.grad under autograd, models/unet_model.py:105), returned as (grads, dx)."""
        grads = OrderedDict()
        dl = np.ascontiguousarray(np.transpose(np.asarray(dlogits_nchw, self.dtype), (0, 2, 3, 1)))
        d, dw, db = conv_valid_bwd(cache["outc.in"], self._w("outc.conv.weight"), dl)
        grads["outc.conv.weight"], grads["outc.conv.bias"] = dw, db
        dskips = {}
        for k in range(4, 0, -1):
            name = f"up{k}"
            dcat = self._double_conv_bwd(_dc_prefix(name), d, cache, grads)
            skip_shape, (oy, ox), cs = cache[name + ".crop"]
            dskip = np.zeros(skip_shape, dtype=self.dtype)
            h, w = dcat.shape[1], dcat.shape[2]
            dskip[:, oy:oy + h, ox:ox + w, :] = self._q(dcat[..., :cs])  # stored bf16 in bf16 plans
            dskips[4 - k] = dskip
            dup = np.ascontiguousarray(dcat[..., cs:])
            d, dw, db = convT2_bwd(self._q(cache[name + ".in"]), self._q(self._w(name + ".up.weight")), self._q(dup))
            if self.gemm == "bf16":
                db = dup.reshape(-1, dup.shape[-1]).sum(0)
            grads[name + ".up.weight"], grads[name + ".up.bias"] = dw, db
        for k in range(4, 0, -1):
            dpool = self._double_conv_bwd(_dc_prefix(f"down{k}"), d, cache, grads)
            arg, in_shape = cache[f"pool{k}"]
            d = maxpool2_bwd(self._q(dpool), arg, in_shape) + dskips[k - 1]
        dx = self._double_conv_bwd(_dc_prefix("inc"), d, cache, grads, need_dx=input_grad)
        if input_grad:
            return grads, np.transpose(dx, (0, 3, 1, 2))
        return grads


def ordered_grads(grads, n_channels=1, n_classes=2):
    """Order a grads dict like model.named_parameters()."""
    return OrderedDict((k, grads[k]) for k in param_shapes(n_channels, n_classes) if not is_buffer(k))


def predict_mask(logits_nchw):
    """scripts/predict.py:85-92: softmax(dim=1)[:,1] > 0.5  ==  logit1 > logit0
    (tie -> background).  Returns uint8 0/255."""
    l = np.asarray(logits_nchw)
    return ((l[:, 1] > l[:, 0]).astype(np.uint8) * 255)


# ----------------------------------------------------------------------------
# Overlap-tile inference geometry (new capability; margin rule of
# scripts/predict1.py:45-46: margin = tile_in - tile_out).
# ----------------------------------------------------------------------------
def overlap_tiles(H, W, tile_in=512):
    """Tiles covering an HxW image with non-overlapping tile_out outputs.

    The image is mirror-padded by margin/2 on the top/left and enough on the
    bottom/right so that every output tile is full.  Returns (tile_out, pad,
    list of (y0, x0) output origins, padded shape)."""
    tile_out = output_size(tile_in)
    m = (tile_in - tile_out) // 2
    ny = -(-H // tile_out)
    nx = -(-W // tile_out)
    pads = (m, ny * tile_out - H + m, m, nx * tile_out - W + m)
    origins = [(ty * tile_out, tx * tile_out) for ty in range(ny) for tx in range(nx)]
    return tile_out, pads, origins


def mirror_pad(img, pads):
    """np.pad(mode='reflect') -- mirror without repeating the edge pixel, the
    overlap-tile strategy of the U-Net paper.  Pads larger than the image are
    reflected repeatedly."""
    top, bottom, left, right = pads
    out = img
    while top or bottom or left or right:
        H, W = out.shape[-2:]
        # a length-1 axis reflects onto itself (np.pad repeats the sample)
        t, b = (top, bottom) if H == 1 else (min(top, H - 1), min(bottom, H - 1))
        l, r = (left, right) if W == 1 else (min(left, W - 1), min(right, W - 1))
        pad = [(0, 0)] * (out.ndim - 2) + [(t, b), (l, r)]
        out = np.pad(out, pad, mode="reflect")
        top, bottom, left, right = top - t, bottom - b, left - l, right - r
    return out
