"""Python handle of a ``unet_plan`` (include/unet_hip.h)."""
from __future__ import annotations

import ctypes

from . import _lib

N_PARAMS = 136   # state_dict entries (parameters + BN buffers)
N_GRADS = 82     # named_parameters
N_SEGMENTS = 9   # backward segments: head+up4, up3, up2, up1, down4, down3, down2, down1, inc
# GEMM arithmetic (include/unet_hip.h UNET_PREC_*): fp32 operands; bf16
# operands with fp32 accumulation (configs C3/C5, torch.autocast(bfloat16));
# fp32-accurate split operands on the bf16 MFMA (hi*hi + hi*lo + lo*hi)
PRECISIONS = {"fp32": 0, "bf16": 1, "bf16x3": 2}


class Plan:
    """One compiled schedule for input shape (n, c, h, w), n_classes and GEMM
    precision ("fp32", "bf16" or "bf16x3")."""

    def __init__(self, n, c, h, w, n_classes, precision="fp32"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
        self.lib = _lib.load()
        self.handle = self.lib.unet_plan_create_ex(n, c, h, w, n_classes, PRECISIONS[precision])
        if not self.handle:
            raise ValueError(f"unet_plan_create_ex({n},{c},{h},{w},{n_classes},{precision}): {_lib.last_error()}")
        self.precision = precision
        oh, ow = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.unet_plan_out_hw(self.handle, ctypes.byref(oh), ctypes.byref(ow)), "unet_plan_out_hw")
        self.shape = (n, c, h, w)
        self.n_classes = n_classes
        self.out_h, self.out_w = oh.value, ow.value
        self.workspace_bytes = int(self.lib.unet_plan_workspace_bytes(self.handle))
        # a forward that no backward follows (eval, no_grad) needs only this prefix
        self.forward_workspace_bytes = int(self.lib.unet_plan_forward_workspace_bytes(self.handle))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self.lib.unet_plan_destroy(h)
            self.handle = None

    def segment_grads(self, seg):
        f, k = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.unet_plan_segment_grads(self.handle, seg, ctypes.byref(f), ctypes.byref(k)),
                   "unet_plan_segment_grads")
        return f.value, k.value

    def forward(self, param_tab, x, logits, ws, train):
        _lib.check(self.lib.unet_plan_forward(self.handle, param_tab, x.data_ptr(), logits.data_ptr(),
                                              ws.data_ptr(), int(bool(train)), _lib.stream_of(x.device)),
                   "unet_plan_forward")

    def backward(self, param_tab, grad_tab, x, dlogits, ws, seg_begin=0, seg_end=N_SEGMENTS, defer_join=False):
        """defer_join: leave the segments' side-stream weight gradients running
        (UNET_BWD_DEFER_JOIN); wait_segment() before reducing a segment's
        gradients and join() before the optimizer."""
        _lib.check(self.lib.unet_plan_backward_ex(self.handle, param_tab, grad_tab, x.data_ptr(), dlogits.data_ptr(),
                                                  ws.data_ptr(), seg_begin, seg_end, 1 if defer_join else 0,
                                                  _lib.stream_of(x.device)),
                   "unet_plan_backward_ex")

    def input_grad(self, param_tab, x, ws):
        """x.grad of the last backward (unet_plan_input_grad): inc.c0's
        BatchNorm-backward output materialised in a scratch tensor, then its
        full correlation with inc.c0's weights.  Same stream as the backward."""
        import torch
        scratch = torch.empty(int(self.lib.unet_plan_input_grad_scratch_bytes(self.handle)), dtype=torch.uint8,
                              device=x.device)
        dx = torch.empty_like(x)
        _lib.check(self.lib.unet_plan_input_grad(self.handle, param_tab, dx.data_ptr(), ws.data_ptr(),
                                                 scratch.data_ptr(), _lib.stream_of(x.device)), "unet_plan_input_grad")
        return dx

    def wait_segment(self, seg, stream):
        """Make `stream` (a torch stream) wait for segment seg's weight gradients."""
        _lib.check(self.lib.unet_plan_wait_segment(self.handle, seg, ctypes.c_void_p(stream.cuda_stream)),
                   "unet_plan_wait_segment")

    def join(self, device):
        """Join the side stream into the current stream of `device`."""
        _lib.check(self.lib.unet_plan_join(self.handle, _lib.stream_of(device)), "unet_plan_join")

    timing_on = False

    def set_timing(self, enable):
        _lib.check(self.lib.unet_plan_set_timing(self.handle, int(bool(enable))), "unet_plan_set_timing")
        self.timing_on = bool(enable)

    def timing(self):
        """{class: (ms, flops, bytes, launches)} accumulated since the last call."""
        n = 6
        ms = (ctypes.c_double * n)()
        fl = (ctypes.c_double * n)()
        by = (ctypes.c_double * n)()
        cnt = (ctypes.c_int * n)()
        _lib.check(self.lib.unet_plan_timing(self.handle, ms, fl, by, cnt), "unet_plan_timing")
        names = ["conv_fwd", "conv_dgrad", "conv_wgrad", "stage1", "elementwise", "bottleneck"]
        return {names[i]: (ms[i], fl[i], by[i], cnt[i]) for i in range(n)}

    def mfma_flops(self):
        """{class: MFMA flops executed} over the intervals of the last timing()
        call (Winograd variants execute fewer than the direct-conv flops)."""
        n = 6
        xf = (ctypes.c_double * n)()
        _lib.check(self.lib.unet_plan_timing_mfma_flops(self.handle, xf), "unet_plan_timing_mfma_flops")
        names = ["conv_fwd", "conv_dgrad", "conv_wgrad", "stage1", "elementwise", "bottleneck"]
        return {names[i]: xf[i] for i in range(n)}

    def timing_sites(self):
        """[(site, ms, direct flops, MFMA flops)] per GEMM launch site of the
        step the last timing() call collected (site = "<layer> <fwd|dgrad|wgrad>")."""
        n = self.lib.unet_plan_timing_sites(self.handle, None, 0)
        buf = ctypes.create_string_buffer(n)
        self.lib.unet_plan_timing_sites(self.handle, buf, n)
        out = []
        for ln in buf.value.decode().splitlines():
            name, ms, fl, xf = ln.split("\t")
            out.append((name, float(ms), float(fl), float(xf)))
        return out
