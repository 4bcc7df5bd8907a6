"""Benchmark: U-Net training images/s at 512x512x1, batch 8 per GPU, fp32
(BASELINE.json configs[1]; weak scaling over 1/2/4/8 MI355X with an RCCL
gradient all-reduce over xGMI).  The same invocation also times the bf16-operand
GEMM plan (configs[2] per GPU: global batch 8 x N) and reports it as the
``bf16`` sub-object; ``--dtype`` picks the precision of the headline ``value``
(default fp32 = configs[1]); ``--channels 3 --size 572`` is the configs[4]
stress shape.

A step = forward + WeightedCrossEntropyLoss + backward + all-reduce (N>1) +
SGD(momentum 0.99) over one synthetic batch resident in HBM, exactly the body
of scripts/train.py:108-131 (no per-step .item()).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE compact JSON line on rank 0 (the contract fields and every headline
number, ~1.5 KB so a 2 KB log tail holds all of it) and writes the full record
-- per-launch-site timings, kernel classes, descriptions -- to --detail-out
(default gpurun_out/bench_detail.json).  The full record carries:
* roofline: the implicit-GEMM conv family (63 GEMM launch sites per step) at
  the MFMA peak of the precision, HIP-event timed on the plan's stream in an
  extra untimed step; `achieved` counts the MFMA flops the chosen variants
  execute (the Winograd layers' point GEMMs), `direct_conv_tflops` the direct
  convolution's flops over the same time; traffic from the committed rocprofv3 PMC passes of this
  command (profiles/pmc_traffic*.json, per GEMM launch site);
* bottleneck / stage1: SURVEY.md §8d's two targets (MFMA on the 1024-channel
  set, HBM on the fused stage-1 kernels);
* iou: eval-mode masks of 12 real DIC-C2DH-HeLa frames (t000-t002 against
  01_ST/SEG, tests/golden/hela_real.npz; the nine gold-truth frames against
  01_GT/SEG, tests/golden/hela_gold.npz), mean IoU next to the reference's on
  the same frames and weights (a checker leg, run after the timing);
* cpu_baseline: the reference train step restated on torch CPU
  (oracle/torch_cpu_ref.py; the reference .py does not travel to the GPU box)
  at batch 8 and batch 1 on this host's cores;
* c5: configs[4] (3-ch 572^2, batch 8, bf16 train step) with its roofline;
  farm: configs[3] (1024^2 overlap-tile inference, fp32 and bf16, one GPU);
* lib: unet_version() with the source hash it was built from, and the tuning
  database replayed (profiles/tune_db.txt: the GEMM choices this line timed,
  loaded by the full-size parity tests too).

value / ms_per_step: the MEDIAN per-step time over the timed steps (HIP events
per step, BASELINE.md's protocol); mean_ms_per_step / wall_value: wall clock.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training images/sec (512×512×1, batch=8) at 1/2/4/8 MI355X; IoU vs ref"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA = f32 vector peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (no sparsity)
HBM_PEAK_GBS = 8000.0
# BASELINE.md:64 asks for fractions against peaks measured on the box as well:
# bench.py measures them in its untimed tail (unet_peak_probe: bf16 / f32 MFMA
# loops, float4 HBM copy) and reports every frac_measured against those.  The
# guide's figures (MI355X_MICROARCH.md: f32 MFMA 155 TF, HBM copy 6.29 TB/s)
# stand in only if the probe fails.
FP32_MFMA_MEASURED_TFLOPS = 155.0
HBM_MEASURED_GBS = 6290.0
BOTTLENECK_LAYERS = ("down4.c0", "down4.c1", "up1.convT", "up1.c0")
GEMM_DESC = {"fp32": "fp32", "bf16": "bf16-operand/fp32-acc",
             "bf16x3": "fp32-accurate bf16x3 split-operand (3 bf16 MFMA products, fp32 acc)"}
PEAK = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS, "bf16x3": round(BF16_MFMA_PEAK_TFLOPS / 3, 1)}
PEAK_MEASURED = {"fp32": FP32_MFMA_MEASURED_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS,
                 "bf16x3": round(BF16_MFMA_PEAK_TFLOPS / 3, 1)}


def init_weights(m):
    """scripts/train.py:54-61."""
    if isinstance(m, torch.nn.Conv2d):
        torch.nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if m.bias is not None:
            torch.nn.init.constant_(m.bias, 0)
    elif isinstance(m, torch.nn.BatchNorm2d):
        torch.nn.init.constant_(m.weight, 1)
        torch.nn.init.constant_(m.bias, 0)


def synthetic_batch(n, size, out, device, seed, channels=1):
    """x ~ U[0,1), target ~ Bernoulli(0.4), weight = 10 + 1/freq(class) per image
    (the committed HeLa weight maps have exactly this form)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.rand((n, channels, size, size), generator=g, device=device)
    t = (torch.rand((n, out, out), generator=g, device=device) < 0.4).long()
    f1 = t.float().mean(dim=(1, 2), keepdim=True).clamp_min(1e-6)
    w = torch.where(t > 0, 10.0 + 1.0 / f1, 10.0 + 1.0 / (1.0 - f1).clamp_min(1e-6))
    return x.contiguous(), t.contiguous(), w.contiguous()


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(steps=5):
    """The reference train step (scripts/train.py:114-131 semantics) restated on
    torch CPU -- the same oneDNN / native kernels the reference runs on -- at
    512x512x1, batch 8 (the metric's batch) and batch 1 (configs[0]), timed on
    this host: `steps` steps per batch size after one warm-up step, images/s
    from the median step.  Measurement infrastructure
    (oracle/torch_cpu_ref.py)."""
    from oracle import torch_cpu_ref as R
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    R.train_steps_per_second(1, seconds=0.0, max_steps=1)
    _, t1 = R.train_step_times(1, steps)
    _, t8 = R.train_step_times(8, steps)
    med = lambda ts: sorted(ts)[len(ts) // 2]  # noqa: E731
    return {"value": round(8 / med(t8), 4), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "batch1_value": round(1 / med(t1), 4),
            "step_s": {"batch8": [round(v, 3) for v in t8], "batch1": [round(v, 3) for v in t1]},
            "sample": f"torch {torch.__version__} CPU restatement of the reference train step (fwd + weighted CE + "
                      f"bwd + SGD(0.99), fp32, 512x512x1): {steps} steps at batch 8 and {steps} at batch 1 after one "
                      f"warm-up step, median step time ({sum(t8) + sum(t1):.1f} s of CPU work)"}


def pmc_traffic(args, dtype):
    """HBM bytes per GEMM launch site and per stage-1 step from the committed PMC
    passes of this command (tools/pmc_report.py --json); counters cannot be read
    in the timed run itself (separate rocprofv3 --pmc passes)."""
    name = "pmc_traffic.json" if dtype == "fp32" else f"pmc_traffic_{dtype}.json"
    path = os.path.join(ROOT, "profiles", name)
    if args.size != 512 or args.batch != 8 or args.channels != 1 or not os.path.exists(path):
        return {}
    return json.load(open(path))


def measure_peaks(device, reps=3):
    """The box's own ceilings (untimed tail, after every timed leg):
    unet_peak_probe kinds 0 / 1 / 2 = dense bf16 MFMA, f32 MFMA (TFLOP/s) and a
    float4 HBM copy (GB/s, read + write bytes), best of `reps` launches."""
    import ctypes
    from unet_amd import _lib
    lib = _lib.load()
    res = {}
    for kind, name in ((0, "bf16_mfma_tflops"), (1, "fp32_mfma_tflops"), (2, "hbm_copy_gbs"), (3, "hbm_read_gbs")):
        v = ctypes.c_double(0.0)
        rc = lib.unet_peak_probe(kind, reps, ctypes.byref(v), _lib.stream_of(device))
        res[name] = round(v.value, 1) if rc == 0 and v.value > 0 else None
    # the HBM ceiling the HBM-bound legs are held against: the higher of the two
    # (the stage-1 kernels read about twice what they write)
    bw = [v for v in (res["hbm_copy_gbs"], res["hbm_read_gbs"]) if v]
    res["hbm_gbs"] = max(bw) if bw else None
    res["method"] = ("unet_peak_probe on this GPU after the timed legs: MFMA loops at 1 and 2 waves per SIMD with "
                     "4-8 independent accumulator chains per wave (v_mfma_f32_32x32x16_bf16; v_mfma_f32_16x16x4_f32 "
                     "and 32x32x2_f32), 32768 iterations; float4 copies of 1 GiB (grid-strided with 1 or 4 loads "
                     "in flight per thread, or one contiguous non-temporal chunk per workgroup) and a 2 GiB "
                     "read-only stream, hbm_gbs = the higher; the best shape, "
                     f"best of {reps} HIP-event-timed launches after a warm-up")
    return res


def apply_measured_peaks(obj, dtype, peaks):
    """Re-express a leg's frac_measured fields against the probed ceilings."""
    mf = {"fp32": peaks.get("fp32_mfma_tflops"), "bf16": peaks.get("bf16_mfma_tflops")}
    mf["bf16x3"] = round(mf["bf16"] / 3, 1) if mf["bf16"] else None
    p, hbm = mf.get(dtype), peaks.get("hbm_gbs")
    rl, bn, st = obj.get("roofline"), obj.get("bottleneck"), obj.get("stage1")
    if p and rl:
        rl["peak_measured"] = p
        rl["frac_measured"] = round(rl["achieved"] / p, 4)
    if p and bn and bn.get("tflops"):
        bn["frac_measured"] = round(bn["tflops"] / p, 4)
    if hbm and st and st.get("achieved_gbs"):
        st["peak_measured_gbs"] = hbm
        st["frac_measured"] = round(st["achieved_gbs"] / hbm, 4)


def compact_line(out, detail):
    """The stdout line: the contract fields plus every headline number (fp32 and
    bf16 values, conv-family and bottleneck fractions, stage 1, c5, farm, IoU,
    CPU baseline, measured peaks), without the per-site tables and prose -- those
    are in the detail file."""
    def pick(d, keys):
        return {k: d[k] for k in keys if d is not None and k in d}

    line = pick(out, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                      "scaling", "vs_baseline", "dtype"))
    line["data"] = "synthetic x~U[0,1), Bernoulli(0.4) targets, 10+1/freq weights, kaiming init"
    line["config"] = {"workload": out["config"]["workload"].split(":")[0] + " (fwd+WCE+bwd+SGD)",
                      **pick(out["config"], ("global_batch", "image", "parallelism"))}
    rl = out["roofline"]
    line["roofline"] = {**pick(rl, ("bound", "achieved", "peak", "unit", "frac", "frac_measured", "traffic")),
                        "kernel": "conv GEMM family (executed MFMA flops)"}
    if "cpu_baseline" in out:
        cb = out["cpu_baseline"]
        line["cpu_baseline"] = {**pick(cb, ("value", "unit", "cores", "kind", "batch1_value")),
                                "sample": "torch-CPU restatement of the reference step, batch 8 / 1, median of 5"}
    line["bottleneck"] = pick(out.get("bottleneck"), ("ms", "frac", "frac_measured"))
    line["stage1"] = pick(out.get("stage1"), ("ms", "achieved_gbs", "frac"))
    for d in ("fp32", "bf16", "bf16x3"):
        if d in out and isinstance(out[d], dict) and "value" in out[d]:
            r = out[d]
            line[d] = {**pick(r, ("value", "ms_per_step")),
                       "frac": r["roofline"]["frac"],
                       "bottleneck": pick(r.get("bottleneck"), ("ms", "frac", "frac_measured")),
                       "elementwise_ms": r.get("kernels", {}).get("elementwise", {}).get("ms")}
            if r.get("iou"):
                line[d]["iou"] = r["iou"]["iou"]
    if "c5" in out:
        line["c5"] = {**pick(out["c5"], ("value", "ms_per_step")), "frac": out["c5"]["roofline"]["frac"],
                      "bottleneck_frac": out["c5"].get("bottleneck", {}).get("frac")}
    if "farm" in out:
        line["farm"] = {d: r["value"] for d, r in out["farm"].items()}
    if out.get("iou"):
        line["iou"] = pick(out["iou"], ("iou", "iou_ref", "frames"))
    if out.get("comm"):
        line["comm"] = pick(out["comm"], ("dtype", "bytes_per_step"))
    if out.get("peaks_measured"):
        line["peaks"] = pick(out["peaks_measured"], ("bf16_mfma_tflops", "fp32_mfma_tflops", "hbm_gbs"))
    line["lib"] = pick(out.get("lib"), ("lib_src", "src_match", "tune_db_entries"))
    if detail:
        line["detail"] = detail
    return line


def hela_frames():
    """The 12 real DIC-C2DH-HeLa 01 frames of the IoU check: t000-t002 with their
    01_ST/SEG masks (tests/golden/hela_real.npz) and the nine gold-truth frames
    t002 ... t067 with 01_GT/SEG (tests/golden/hela_gold.npz), the eval model's
    weights (hash init + the running statistics of hela_real.npz) and the
    reference's IoU per frame.  None if the fixtures are absent."""
    import numpy as np
    from oracle import unet_oracle as O
    pr, pg = (os.path.join(ROOT, "tests", "golden", f) for f in ("hela_real.npz", "hela_gold.npz"))
    if not (os.path.exists(pr) and os.path.exists(pg)):
        return None
    zr, zg = np.load(pr, allow_pickle=False), np.load(pg, allow_pickle=False)
    params = O.hash_init(1, 2, seed=int(zr["seed"]), bn_random=True)
    for k in zr.files:
        if k.startswith("buf/"):
            params[k[4:]] = zr[k].astype(np.float32)
    images = np.concatenate([zr["images"], zg["images"]])
    fg = np.concatenate([zr["segs"] > 0, np.unpackbits(zg["seg_fg"], axis=-1)[..., :512].astype(bool)])
    names = [f"ST t{i:03d}" for i in range(len(zr["images"]))] + [f"GT t{int(i):03d}" for i in zg["frames"]]
    return params, images, fg, np.concatenate([zr["ious"], zg["ious"]]), names


def hela_iou(device, precision):
    """Checker leg (after the timing): eval-mode masks of the 12 real HeLa frames
    of hela_frames() vs their segmentations, next to the reference's IoUs on the
    same frames and weights (utils/metrics.py:6-37)."""
    import numpy as np
    from unet_amd import UNet, _lib
    fr = hela_frames()
    if fr is None:
        return None
    params, images, fg, ref, _ = fr
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.to(device).eval()
    m.precision = precision
    x = torch.from_numpy((images.astype(np.float32)[:, None] / 255.0) * 2.0 - 1.0).to(device)
    with torch.no_grad():
        logits = m(x)
    lib = _lib.load()
    n, _, oh, ow = logits.shape
    mask = torch.empty((n, oh, ow), dtype=torch.uint8, device=device)
    _lib.check(lib.unet_mask_from_logits(logits.data_ptr(), mask.data_ptr(), n, oh, ow, _lib.stream_of(device)),
               "unet_mask_from_logits")
    oy = (fg.shape[1] - oh) // 2
    gt = torch.from_numpy(fg[:, oy:oy + oh, oy:oy + ow].astype(np.uint8) * 255).to(device)
    ious = []
    for i in range(n):
        cnt = torch.zeros(2, dtype=torch.int64, device=device)
        _lib.check(lib.unet_iou_counts(mask[i].data_ptr(), gt[i].contiguous().data_ptr(), oh * ow, cnt.data_ptr(),
                                       _lib.stream_of(device)), "unet_iou_counts")
        c = cnt.cpu().numpy()
        ious.append(float(c[0] / c[1]) if c[1] else 1.0)
    ref = [float(v) for v in ref]
    return {"iou": round(float(np.mean(ious)), 6), "iou_ref": round(float(np.mean(ref)), 6),
            "max_abs_diff": float(max(abs(a - b) for a, b in zip(ious, ref))), "frames": n,
            "data": "DIC-C2DH-HeLa 01: t000-t002 vs 01_ST/SEG and the nine gold-truth frames t002, t005, t021, t031, "
                    "t033, t034, t039, t054, t067 vs 01_GT/SEG, eval mode, Normalize(0.5, 0.5) (predict.py:50-92); "
                    "iou_ref = the reference UNet on the same frames and weights (tests/golden/hela_real.npz, "
                    "hela_gold.npz)"}


def run_farm(args, dtype, device, iters=20, warmup=3):
    """configs[3] on one GPU: overlap-tile inference of a 1024x1024 image as
    16 tiles of 512x512 (324x324 out), batch 8, eval mode, uint8 mask out
    (scripts/predict.py:70-92 per tile; unet_amd/tiling.py).  Tiles farm over N
    GPUs with no collective (replicas), so N GPUs scale this by N."""
    from unet_amd import UNet
    from unet_amd.tiling import TileFarm, TileGeometry
    torch.manual_seed(0)
    m = UNet(1, 2)
    m.apply(init_weights)
    m.precision = dtype
    farm = TileFarm(m, devices=[device.index], tile_in=512, batch=8)
    for r in farm.replicas:
        r.precision = dtype
    g = torch.Generator().manual_seed(5)
    img = torch.rand((1, 1024, 1024), generator=g) * 2 - 1
    for _ in range(warmup):
        farm.predict(img, return_mask=True)
    torch.cuda.synchronize()
    times = []
    for _ in range(iters):
        t0 = time.perf_counter()
        mask = farm.predict(img, return_mask=True)   # includes the host copy of the mask
        times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    geo = TileGeometry(1024, 1024, 512)
    return {"value": round(1 / med, 3), "unit": "images/s", "ms_per_image": round(med * 1e3, 3),
            "tiles_per_s": round(len(geo) / med, 1), "dtype": dtype,
            "config": {"workload": "overlap-tile inference 1024x1024x1 (configs[3]), 512^2 tiles -> 324^2, "
                                   f"{len(geo)} tiles, batch 8, eval mode, mask output, measured on 1 GPU (the farm deals tiles to per-GPU replicas with no exchange; multi-GPU farm throughput is not measured here)",
                       "mask_shape": list(mask.shape)}}


def run_precision(args, dtype, device, pg, world, rank):
    """Time args.steps train steps of one GEMM precision; returns its summary.
    UNET_MAIN_PRIORITY=<p> (experiment): the whole leg runs on a torch stream
    of priority p (lower = higher), the plan's side stream keeps the lowest."""
    prio = os.environ.get("UNET_MAIN_PRIORITY")
    if not prio:
        return _run_precision(args, dtype, device, pg, world, rank)
    s = torch.cuda.Stream(device=device, priority=int(prio))
    print(f"main stream priority {int(prio)} (range {torch.cuda.Stream.priority_range()})", file=sys.stderr)
    torch.cuda.current_stream(device).synchronize()
    with torch.cuda.stream(s):
        r = _run_precision(args, dtype, device, pg, world, rank)
    s.synchronize()
    return r


def _run_precision(args, dtype, device, pg, world, rank):
    from unet_amd import UNet
    from unet_amd.train import Trainer
    torch.manual_seed(0)
    model = UNet(n_channels=args.channels, n_classes=2)
    model.apply(init_weights)
    model = model.to(device).train()
    if pg is not None:  # identical start on every rank
        for t in model.state_dict().values():
            dist.broadcast(t, 0)
    trainer = Trainer(model, args.batch, args.size, args.size, lr=1e-4, momentum=0.99, process_group=pg,
                      overlap=not args.no_overlap, precision=dtype, graph=args.graph)
    oh, ow = trainer.out_hw
    x, t, w = synthetic_batch(args.batch, args.size, oh, device, seed=1234 + rank, channels=args.channels)

    for _ in range(args.warmup):
        trainer.step(x, t, w)
    torch.cuda.synchronize()
    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step HIP events on the stream every step joins into (the side stream
    # and the collectives are waited on before the optimizer): the median step
    # (BASELINE.md protocol) next to the wall-clock mean; no host sync inside
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        loss = trainer.step(x, t, w)
        evs[i + 1].record()
    torch.cuda.synchronize()
    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    median_ms = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else 0.5 * (step_ms[len(step_ms) // 2 - 1] +
                                                                              step_ms[len(step_ms) // 2])
    if pg is not None:
        e = torch.tensor([elapsed, median_ms], dtype=torch.float64, device=device)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed, median_ms = float(e[0].item()), float(e[1].item())
    final_loss = float(loss.item())

    # per-kernel-class timing of one extra (untimed) step: HIP events recorded by
    # the plan on the stream its kernels run on
    trainer.plan.set_timing(True)
    trainer.step(x, t, w)
    torch.cuda.synchronize()
    trainer.plan.set_timing(False)
    tim = trainer.plan.timing()
    xfl = trainer.plan.mfma_flops()
    sites = trainer.plan.timing_sites()
    comm = None
    if pg is not None:
        comm = {"collective": f"all_reduce(SUM) of {len(trainer.reducer.buckets)} gradient buckets, each issued as its "
                              "backward segment finishes" if trainer.overlap else "one all_reduce after backward",
                "dtype": str(trainer.comm_dtype).replace("torch.", ""),
                "bytes_per_step": trainer.reducer.bytes_per_step,
                "buffers": "rank 0's BatchNorm running statistics (one flat buffer) as each forward left them, "
                           "broadcast beside that step's backward and applied at the next step's start"}
    del trainer, model, x, t, w
    torch.cuda.empty_cache()

    peak, peak_m = PEAK[dtype], PEAK_MEASURED[dtype]
    conv = [tim[k] for k in ("conv_fwd", "conv_dgrad", "conv_wgrad")]
    conv_ms = sum(c[0] for c in conv)
    conv_fl = sum(c[1] for c in conv)
    launches = sum(c[3] for c in conv)
    conv_xfl = sum(xfl[k] for k in ("conv_fwd", "conv_dgrad", "conv_wgrad"))
    # roofline: MFMA flops the GEMMs execute (Winograd layers run 2.25x / 4x fewer
    # than the direct convolution); the direct-convolution rate beside it
    achieved = conv_xfl / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
    direct = conv_fl / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
    pmc = pmc_traffic(args, dtype)
    fam = pmc.get("families", {})
    st, bn = tim["stage1"], tim["bottleneck"]
    kernels = {k: {"ms": round(v[0], 3), "launches": v[3],
                   "tflops": round(v[1] / (v[0] * 1e-3) / 1e12, 2) if v[0] > 0 and v[1] else None,
                   "mfma_tflops": round(xfl[k] / (v[0] * 1e-3) / 1e12, 2) if v[0] > 0 and xfl[k] else None,
                   "gbs": round(v[2] / (v[0] * 1e-3) / 1e9, 1) if v[0] > 0 and v[2] else None}
               for k, v in tim.items()}
    imgs = world * args.batch * args.steps
    return {
        # images/s = world * batch / median step time
        "value": round(world * args.batch / (median_ms * 1e-3), 3),
        "ms_per_step": round(median_ms, 3),
        "mean_ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "wall_value": round(imgs / elapsed, 3),
        "step_ms_range": [round(step_ms[0], 3), round(step_ms[-1], 3)],
        "dtype": dtype,
        "roofline": {"bound": "mfma", "kernel": f"implicit-GEMM conv family (fwd/dgrad igemm + wgrad, {dtype} operands)",
                     "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4),
                     "peak_measured": peak_m, "frac_measured": round(achieved / peak_m, 4),
                     "traffic": fam.get("conv", {}).get("bytes_per_launch"),
                     "traffic_unit": ("HBM bytes per GEMM launch site (rocprofv3 --pmc 2*FETCH_SIZE + WRITE_SIZE of "
                                      "this command's conv family incl. split-K epilogues, summed over one step / "
                                      f"{launches}; profiles/pmc_traffic{'' if dtype == 'fp32' else '_' + dtype}.json)"
                                      if fam.get("conv") else None),
                     "flops": "MFMA flops the chosen GEMM variants execute (Winograd F(2x2,3x3) / F(4x4,3x3) "
                              "point GEMMs: 2 x points x tiles x Cin x Cout; else the direct 2 x M x N x K)",
                     "mfma_flops_per_step": conv_xfl,
                     "direct_conv_flops_per_step": conv_fl,
                     "direct_conv_tflops": round(direct, 2),
                     "launches_per_step": launches,
                     "avg_launch_ms": round(conv_ms / max(launches, 1), 4),
                     "timing": "HIP events on the plan's stream over one extra step after the timed steps, "
                               "weight-gradient side stream serialised; in the timed steps wgrad overlaps dgrad "
                               "on a second stream (per-dispatch times then overlap: profiles/*trace_check*.txt)"},
        # SURVEY.md §8d target: >= 50 % MFMA on the 1024-channel bottleneck set
        "bottleneck": {"layers": "down4.c0, down4.c1, up1.convT, up1.c0 (fwd + dgrad + wgrad)",
                       "ms": round(bn[0], 3),
                       "tflops": round(xfl["bottleneck"] / (bn[0] * 1e-3) / 1e12, 2) if bn[0] > 0 else None,
                       "frac": round(xfl["bottleneck"] / (bn[0] * 1e-3) / 1e12 / peak, 4) if bn[0] > 0 else None,
                       "frac_measured": round(xfl["bottleneck"] / (bn[0] * 1e-3) / 1e12 / peak_m, 4)
                       if bn[0] > 0 else None,
                       "direct_conv_tflops": round(bn[1] / (bn[0] * 1e-3) / 1e12, 2) if bn[0] > 0 else None,
                       # per launch site: ms and executed-MFMA TFLOP/s (the split of the set)
                       "sites": {nm: [round(ms, 4), round(xf / (ms * 1e-3) / 1e12, 1) if ms > 0 else None]
                                 for nm, ms, _, xf in sites if nm.split(" ")[0] in BOTTLENECK_LAYERS}},
        # every GEMM launch site of the timing step: [ms, executed-MFMA TFLOP/s]
        "gemm_sites": {nm: [round(ms, 4), round(xf / (ms * 1e-3) / 1e12, 1) if ms > 0 else None]
                       for nm, ms, _, xf in sites},
        # SURVEY.md §8d target: >= 40 % HBM on stage 1 (inc.c0 + BN0 stats fwd;
        # BN0 backward fused into inc.c0's weight gradient)
        "stage1": {"bound": "hbm", "ms": round(st[0], 3), "launches": st[3],
                   "kernels": "k_conv_first_fwd (read x, write y0, BN0 stats) + k_bnb_finalize(BN0) + "
                              "k_conv_first_wgrad<FUSED> (read dz0, y0, x) + k_reduce_slabs",
                   "algorithmic_bytes": st[2],
                   "achieved_gbs": round(st[2] / (st[0] * 1e-3) / 1e9, 1) if st[0] > 0 else None,
                   "peak_gbs": HBM_PEAK_GBS,
                   "frac": round(st[2] / (st[0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if st[0] > 0 else None,
                   "peak_measured_gbs": HBM_MEASURED_GBS,
                   "frac_measured": round(st[2] / (st[0] * 1e-3) / 1e9 / HBM_MEASURED_GBS, 4) if st[0] > 0 else None,
                   "traffic": fam.get("stage1", {}).get("bytes_per_step")},
        "kernels": kernels,
        "final_loss": round(final_loss, 5),
        "comm": comm,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--channels", type=int, default=1, help="input channels (configs[4]: 3)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "bf16x3"],
                    help="GEMM arithmetic of the headline value: fp32 MFMA; bf16 = bf16-in / fp32-acc MFMA; "
                         "bf16x3 = fp32-accurate split operands (hi*hi + hi*lo + lo*hi on the bf16 MFMA)")
    ap.add_argument("--extra-dtypes", default="bf16",
                    help="comma-separated precisions also timed in this invocation and reported as sub-objects "
                         "('' = none; profiling runs use '')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-iou", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="single process: replay the whole train step as one hipGraph after the autotuned warm-up")
    ap.add_argument("--tuning-report", default=None, help="write the GEMM autotuner's choices to this file")
    ap.add_argument("--tune-db", default=os.path.join(ROOT, "profiles", "tune_db.txt"),
                    help="GEMM choices to replay (the committed database the full-size tests load too); shapes it "
                         "does not hold are tuned live")
    ap.add_argument("--retune", action="store_true", help="ignore --tune-db: time every GEMM variant afresh")
    ap.add_argument("--tune-db-out", default=None, help="save the process's GEMM choices to this file at the end")
    ap.add_argument("--no-extras", action="store_true", help="skip the farm (configs[3]) and c5 (configs[4]) legs")
    ap.add_argument("--no-peaks", action="store_true", help="skip the untimed peak probes of the tail")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, one GPU per rank) or gloo (ranks may share a GPU; rehearsal only)")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="write the full record (per-site timings, kernel classes) here ('' = don't)")
    ap.add_argument("--full-stdout", action="store_true", help="print the full record instead of the compact line "
                    "(tools that read kernel classes from stdout)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; "--dist-backend gloo" lets several ranks share a device
    # (a rehearsal of the DP path on a 1-GPU box, not a measurement)
    local_dev = local if args.dist_backend == "nccl" else local % torch.cuda.device_count()
    torch.cuda.set_device(local_dev)
    device = torch.device("cuda", local_dev)
    pg = None
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)
        pg = dist.group.WORLD

    from unet_amd import _lib as _ulib
    lib = _ulib.load()
    ident = _ulib.build_identity()
    tune_db_entries = 0
    if not args.retune and args.tune_db and os.path.exists(args.tune_db):
        tune_db_entries = lib.unet_tuning_load(args.tune_db.encode())
        if tune_db_entries < 0:
            raise RuntimeError(f"unet_tuning_load({args.tune_db}) failed: {tune_db_entries}")

    main_res = run_precision(args, args.dtype, device, pg, world, rank)
    extras = {}
    for d in [d for d in args.extra_dtypes.split(",") if d and d != args.dtype]:
        extras[d] = run_precision(args, d, device, pg, world, rank)
    farm, c5 = {}, None
    if not args.no_extras and args.size == 512 and args.channels == 1 and args.batch == 8:
        # configs[4]: 3-ch 572^2, batch 8 per GPU, bf16 train step
        c5_args = argparse.Namespace(**{**vars(args), "channels": 3, "size": 572,
                                        "steps": max(5, args.steps // 2), "warmup": max(3, args.warmup // 2)})
        c5 = run_precision(c5_args, "bf16", device, pg, world, rank)
        c5["steps"] = c5_args.steps
        if world == 1:  # configs[3] farms tiles over GPUs with no collective: one GPU's rate x N
            for d in ("fp32", "bf16"):
                farm[d] = run_farm(args, d, device)

    if rank == 0:
        comm = f" + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} all-reduce" if world > 1 else ""
        out = {
            "metric": METRIC,
            "value": main_res["value"],
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": f"synthetic: x~U[0,1) (N,{args.channels},{args.size},{args.size}), Bernoulli(0.4) targets, "
                    "10+1/freq(class) weight maps; kaiming fan_out init (scripts/train.py:54-61)",
            "config": {"workload": f"U-Net train step {args.size}x{args.size}x{args.channels}, batch {args.batch}/GPU, "
                                   f"{GEMM_DESC[args.dtype]} GEMMs: fwd + weighted CE + bwd + SGD(0.99){comm}",
                       "global_batch": world * args.batch, "image": args.size,
                       "parallelism": f"dp{world}"},
        }
        for k in ("mean_ms_per_step", "wall_value", "step_ms_range", "roofline", "bottleneck", "stage1", "kernels",
                  "gemm_sites", "final_loss"):
            out[k] = main_res[k]
        out["lib"] = {**ident, "tune_db": os.path.relpath(args.tune_db, ROOT) if tune_db_entries > 0 else None,
                      "tune_db_entries": tune_db_entries}
        if main_res["comm"] is not None:
            out["comm"] = main_res["comm"]
        for d, r in extras.items():
            out[d] = {"value": r["value"], "unit": "images/s", "ms_per_step": r["ms_per_step"],
                      "mean_ms_per_step": r["mean_ms_per_step"],
                      "config": f"same workload, {GEMM_DESC[d]} GEMMs (global batch {world * args.batch}"
                                f"{'; configs[2] at N=8' if d == 'bf16' else ''})",
                      **{k: r[k] for k in ("roofline", "bottleneck", "stage1", "kernels", "gemm_sites", "final_loss")}}
        if c5 is not None:
            out["c5"] = {"value": c5["value"], "unit": "images/s", "ms_per_step": c5["ms_per_step"],
                         "steps": c5["steps"], "dtype": "bf16",
                         "config": f"configs[4]: U-Net train step 572x572x3 (388x388 out), batch {args.batch}/GPU, "
                                   "bf16-operand/fp32-acc GEMMs: fwd + weighted CE + bwd + SGD(0.99), synthetic",
                         **{k: c5[k] for k in ("roofline", "bottleneck", "kernels", "final_loss")}}
            if out["c5"]["roofline"].get("traffic") is None:  # no PMC pass of the 572^2 shape is committed
                for k in ("traffic", "traffic_unit"):
                    out["c5"]["roofline"].pop(k, None)
        if farm:
            out["farm"] = farm
        if args.tuning_report:
            with open(args.tuning_report, "w") as f:
                f.write(_ulib.tuning_report())
        if args.tune_db_out:
            lib.unet_tuning_save(args.tune_db_out.encode())
        if not args.no_iou and args.channels == 1:
            out["iou"] = hela_iou(device, args.dtype)
            if "bf16" in extras and out["iou"] is not None:
                out["bf16"]["iou"] = hela_iou(device, "bf16")
        if world == 1 and not args.no_cpu_baseline and args.channels == 1:
            out["cpu_baseline"] = cpu_baseline()
        if not args.no_peaks:
            peaks = measure_peaks(device)
            out["peaks_measured"] = peaks
            apply_measured_peaks(out, args.dtype, peaks)
            for d in extras:
                apply_measured_peaks(out[d], d, peaks)
            if "c5" in out:
                apply_measured_peaks(out["c5"], "bf16", peaks)
        # the full record (every GEMM launch site, kernel classes, descriptions)
        # goes to a file; stdout carries one compact line that fits a 2 KB log
        # tail with every headline in it
        detail = args.detail_out
        if detail:
            os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(out, f, indent=1)
        print(json.dumps(out) if args.full_stdout else json.dumps(compact_line(out, detail), separators=(",", ":")))
    if pg is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
