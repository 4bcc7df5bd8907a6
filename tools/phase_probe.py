"""Phase timeline of k_conv3_bf (tile 31) from a diagnosis build (-DUNET_PHASE_PROBE:
igemm_bf16.hip compiled with it, see igemm_bf16.hip UNET_PROBE).

    python tools/phase_probe.py [--shape inc.c1] [--dgrad] [--variant 31]

Runs the per-op bf16 conv (op_a16) once after warm-ups, reads every workgroup's
s_memrealtime stamps (100 MHz) and prints the median / p90 phase durations:
0 start -> 1 first chunk staged -> 2 chunk-0 MFMAs -> 3 chunk-1 staged ->
4 chunk-1 MFMAs -> 5 loop end -> 6 epilogue end, plus workgroups resident per CU.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from unet_amd import _lib  # noqa: E402
from conv_bench import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="inc.c1")
    ap.add_argument("--dgrad", action="store_true")
    ap.add_argument("--variant", type=int, default=31)
    args = ap.parse_args()
    lib = _lib.load()
    lib.unet_phase_probe_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.unet_set_tuning(b"op_precision", 1)
    lib.unet_set_tuning(b"op_a16", 1)
    lib.unet_set_tuning(b"igemm_variant", args.variant)
    _, n, h, w, ci, co = [s for s in SHAPES if s[0] == args.shape][0]
    dev = "cuda"
    x = torch.randn(n, h, w, ci, device=dev)
    wt = torch.randn(co, ci, 3, 3, device=dev) / (9 * ci) ** 0.5
    b = torch.randn(co, device=dev)
    y = torch.empty(n, h - 2, w - 2, co, device=dev)
    dy = torch.randn(n, h - 2, w - 2, co, device=dev)
    dx = torch.empty(n, h, w, ci, device=dev)
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        if args.dgrad:
            rc = lib.unet_conv3x3_dgrad(dy.data_ptr(), n, h, w, ci, wt.data_ptr(), co, dx.data_ptr(), ws.data_ptr(), st)
        else:
            rc = lib.unet_conv3x3_fwd(x.data_ptr(), n, h, w, ci, wt.data_ptr(), b.data_ptr(), co, None, None,
                                      y.data_ptr(), ws.data_ptr(), st)
        assert rc == 0, rc

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    assert lib.unet_phase_probe_clear() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros((1 << 14, 8), dtype=np.uint64)
    assert lib.unet_phase_probe_read(buf.ctypes.data, buf.nbytes) == 0
    used = buf[:, 0] != 0
    t = buf[used, :7].astype(np.int64)
    ids = buf[used, 7]
    nwg = int(used.sum())
    print(f"{args.shape} {'dgrad' if args.dgrad else 'fwd'} variant {args.variant}: {nwg} workgroups probed, "
          f"launch (op total incl. packing) {e0.elapsed_time(e1) * 1e3:.0f} us")
    t0 = t[:, 0].min()
    span = (t[:, 6].max() - t0) / 100.0
    print(f"probed span first start -> last end: {span:.1f} us")
    names = ["stage0", "mfma0", "stage1", "mfma1", "loopend", "epilogue"]
    prev = t[:, 0]
    for k, nm in enumerate(names, start=1):
        cur = t[:, k]
        ok = cur > 0
        d = (cur[ok] - prev[ok]) / 100.0
        if ok.any():
            print(f"  {nm:9s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f} us  (n={int(ok.sum())})")
            prev = np.where(ok, cur, prev)
    tot = (t[:, 6] - t[:, 0]) / 100.0
    print(f"  total     median {np.median(tot):7.2f} us  p90 {np.percentile(tot, 90):7.2f} us")
    # residency: workgroups per (xcc, se, cu) over time
    hw = ids & 0xFFFFFFFF
    xcc = (ids >> 32) & 0xF
    cu = ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4) | ((hw >> 12) & 1) << 7
    key = xcc * 256 + cu
    conc = []
    for kk in np.unique(key)[:64]:
        sel = key == kk
        s0, s1 = t[sel, 0], t[sel, 6]
        ev = sorted([(a, 1) for a in s0] + [(b, -1) for b in s1])
        c = m = 0
        for _, dd in ev:
            c += dd
            m = max(m, c)
        conc.append(m)
    print(f"  max workgroups resident per CU (64 CUs sampled): median {np.median(conc):.0f}, max {max(conc)}")
    print(f"  CUs seen: {len(np.unique(key))}")


if __name__ == "__main__":
    main()
