"""A/B timing of the bf16 3x3-conv GEMM variants through the per-op C-ABI.

    python tools/conv_bench.py [--reps 20]

For U-Net layer shapes (batch 8, 512x512 input) it times unet_conv3x3_fwd /
unet_conv3x3_dgrad with op_precision=bf16 and each forced igemm variant
(-1 = built-in choice, 21-26 row gather, 31-36 halo, 41-44 persistent halo),
interleaved in one process (rule: perf deltas from interleaved rounds), and
prints the median microseconds and TFLOP/s per variant.
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))
from unet_amd import _lib  # noqa: E402

# (name, n, h, w, ci, co): conv input grid h x w (output h-2 x w-2)
SHAPES = [
    ("inc.c1", 8, 510, 510, 64, 64),
    ("down1.c1", 8, 252, 252, 128, 128),
    ("down2.c1", 8, 123, 123, 256, 256),
    ("down3.c1", 8, 58, 58, 512, 512),
    ("down4.c1", 8, 26, 26, 1024, 1024),
    ("up1.c0", 8, 48, 48, 1024, 512),
    ("up2.c0", 8, 88, 88, 512, 256),
    ("up3.c0", 8, 168, 168, 256, 128),
    ("up4.c0", 8, 328, 328, 128, 64),
    ("up4.c1", 8, 326, 326, 64, 64),
]
VARIANTS = [-1, 21, 22, 23, 24, 31, 32, 33, 34, 35, 36, 41, 42, 43, 44]
DMA_VARIANTS = [31, 33, 63, 65, 66, 67, 68]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dgrad", action="store_true")
    ap.add_argument("--wgrad", action="store_true", help="time the weight gradient over wgrad variants")
    ap.add_argument("--prec", type=int, default=1, help="0 = fp32, 1 = bf16 operands, 2 = bf16x3 split operands")
    ap.add_argument("--a16", action="store_true", help="bf16-stored A as in a bf16 plan (op_a16; tiles 61-66)")
    ap.add_argument("--variants", default=None, help="comma-separated variant ids")
    ap.add_argument("--shapes", default=None, help="comma-separated shape names")
    ap.add_argument("--no-tf", action="store_true",
                    help="forward without the consumer BN+ReLU (the bf16 plan's normalised-copy operand; ring tiles)")
    args = ap.parse_args()
    lib = _lib.load()
    lib.unet_set_tuning(b"op_precision", args.prec)
    lib.unet_set_tuning(b"op_a16", int(args.a16))
    variants = {0: [-1, 1, 2, 3, 4, 8, 11, 12, 13, 14, 51, 52, 53, 54], 1: VARIANTS,
                2: [-1, 21, 22, 23, 24, 25, 26, 31, 33, 35]}[args.prec]
    if args.a16:
        variants = DMA_VARIANTS
    if args.variants:
        variants = [int(v) for v in args.variants.split(",")]
    knob = b"igemm_variant"
    if args.wgrad:  # -1 built-in; fp32 22/23 halo; bf16 / bf16x3 10-14 pixel-column, 20/21 halo,
        # 24/25 wide halo, 26-31 LDS-DMA ring (bf16-stored operands: --a16)
        knob = b"wgrad_variant"
        variants = [-1, 1, 22, 23] if args.prec == 0 else [-1, 10, 12, 13, 20, 21]
        if args.variants:
            variants = [int(v) for v in args.variants.split(",")]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, n, h, w, ci, co in SHAPES:
        if args.shapes and name not in args.shapes.split(","):
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn((n, h, w, ci), device="cuda", generator=g)
        wt = torch.randn((co, ci, 3, 3), device="cuda", generator=g) / (3 * ci ** 0.5)
        b = torch.randn(co, device="cuda", generator=g)
        sc = torch.rand(ci, device="cuda", generator=g) + 0.5
        sh = torch.randn(ci, device="cuda", generator=g) * 0.1
        y = torch.empty((n, h - 2, w - 2, co), device="cuda")
        dy = torch.randn((n, h - 2, w - 2, co), device="cuda", generator=g)
        dx = torch.empty((n, h, w, ci), device="cuda")
        ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
        flops = 2.0 * n * (h - 2) * (w - 2) * ci * co * 9

        dw = torch.empty((co, ci, 3, 3), device="cuda")
        db = torch.empty(co, device="cuda")

        def run():
            if args.wgrad:
                rc = lib.unet_conv3x3_wgrad(x.data_ptr(), dy.data_ptr(), n, h, w, ci, co, dw.data_ptr(),
                                            db.data_ptr(), ws.data_ptr(), st)
            elif args.dgrad:
                rc = lib.unet_conv3x3_dgrad(dy.data_ptr(), n, h, w, ci, wt.data_ptr(), co, dx.data_ptr(),
                                            ws.data_ptr(), st)
            else:
                rc = lib.unet_conv3x3_fwd(x.data_ptr(), n, h, w, ci, wt.data_ptr(), b.data_ptr(), co,
                                          None if args.no_tf else sc.data_ptr(), None if args.no_tf else sh.data_ptr(),
                                          y.data_ptr(), ws.data_ptr(), st)
            return rc

        times = {v: [] for v in variants}
        ok = {}
        for v in variants:
            lib.unet_set_tuning(knob, v)
            ok[v] = run() == 0
        torch.cuda.synchronize()
        for _ in range(args.reps):
            for v in variants:
                if not ok[v]:
                    continue
                lib.unet_set_tuning(knob, v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1e3)
        line = f"{name:9s} {'wgrad' if args.wgrad else 'dgrad' if args.dgrad else 'fwd':5s}"
        for v in variants:
            if ok[v]:
                t = sorted(times[v])[len(times[v]) // 2]
                line += f" | {v}:{t:7.1f}us {flops / t / 1e6:6.1f}TF"
        print(line, flush=True)
    lib.unet_set_tuning(b"igemm_variant", -1)
    lib.unet_set_tuning(b"wgrad_variant", -1)
    lib.unet_set_tuning(b"op_precision", 0)
    lib.unet_set_tuning(b"op_a16", 0)


if __name__ == "__main__":
    main()
