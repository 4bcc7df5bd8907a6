"""fp32 accuracy ablation at configs[1]'s image size.

One process: the reference's arithmetic on torch CPU in fp64 and fp32
(oracle/torch_cpu_ref.py, batch 2 x 512^2, the seed of
tests/golden/train_n2_512.npz), then one GPU train step (drop-in UNet +
WeightedCrossEntropyLoss) per GEMM configuration, each with a fresh tuning
cache.  Per configuration it prints the logits error, the BatchNorm running
variance error per layer (= the batch variance's error x momentum), and the
gradient tensors with the largest rel-L2 error against their bar of
test_fp32_512_every_logit_and_gradient_vs_reference_fp64 (max(1 %, 2 x the
fp32 reference's own error)).

    python tools/acc512.py [config ...]
config: name=knob:value,knob:value  (unet_set_tuning knobs; 'db' loads
profiles/tune_db.txt first), e.g.  direct=wino_max:0,wino_dgrad_max:0
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))
from oracle import fixtures as F  # noqa: E402
from oracle import torch_cpu_ref as R  # noqa: E402
from oracle import unet_oracle as O  # noqa: E402

DEFAULTS = {"wino_max": 4, "wino_dgrad_max": 4, "wino_wgrad_max": 6, "wino4_fwd_min_cg": 128,
            "force_split": 0, "force_tile": 0, "autotune": 1}

CONFIGS = [
    "db=db",
    "live=",
    "f4all=wino4_fwd_min_cg:0",
    "direct=wino_max:0,wino_dgrad_max:0",
    "split2=force_split:2",
    "split4=force_split:4",
    "split8=force_split:8",
]


def torch_ref(params, x, tgt, wmap, dtype):
    net = R.TorchCpuUNet(params, dtype=dtype)
    lg = net.forward(torch.from_numpy(x).to(dtype))
    loss = R.weighted_ce(lg, torch.from_numpy(tgt), torch.from_numpy(wmap).to(dtype))
    loss.backward()
    grads = {k: v.grad.double().numpy() for k, v in net.p.items() if v.requires_grad}
    bufs = {k: v.double().numpy() for k, v in net.p.items() if O.is_buffer(k) and v.is_floating_point()}
    return lg.detach().double().numpy(), float(loss.item()), grads, bufs


def main():
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfgs = sys.argv[1:] or CONFIGS
    z = np.load(os.path.join(ROOT, "tests", "golden", "train_n2_512.npz"), allow_pickle=False)
    seed, n, h = int(z["x_seed"]), int(z["n"]), int(z["h"])
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h)
    t0 = time.time()
    rl, rloss, rg, rb = torch_ref(params, x, tgt, wmap, torch.float64)
    _, _, r32, rb32 = torch_ref(params, x, tgt, wmap, torch.float32)
    print(f"torch CPU fp64 + fp32 reference: {time.time() - t0:.1f} s", flush=True)
    from unet_amd import UNet, WeightedCrossEntropyLoss, _lib
    lib = _lib.load()
    for cfg in cfgs:
        name, _, spec = cfg.partition("=")
        knobs = dict(DEFAULTS)
        use_db = False
        for kv in filter(None, spec.split(",")):
            if kv == "db":
                use_db = True
                continue
            k, v = kv.split(":")
            knobs[k] = int(v)
        lib.unet_tuning_reset()
        for k, v in knobs.items():
            lib.unet_set_tuning(k.encode(), v)
        if use_db:
            lib.unet_tuning_load(os.path.join(ROOT, "profiles", "tune_db.txt").encode())
        m = UNet(1, 2)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
        m = m.cuda().train()
        logits = m(torch.from_numpy(x).cuda())
        loss = WeightedCrossEntropyLoss()(logits, torch.from_numpy(tgt).cuda(), torch.from_numpy(wmap).cuda())
        loss.backward()
        torch.cuda.synchronize()
        lg = logits.detach().double().cpu().numpy()
        print(f"== {name} {spec}: logits max|err| {np.abs(lg - rl).max():.2e}, loss rel {abs(loss.item() - rloss) / rloss:.2e}")
        sd = m.state_dict()
        vrow = []
        for k in rb:
            if not k.endswith("running_var"):
                continue
            # running_var = 0.9 rv0 + 0.1 var_b: error / 0.1 is the batch variance's
            r0 = np.asarray(params[k], np.float64)
            vb = (rb[k] - 0.9 * r0) / 0.1
            eg = np.abs((sd[k].double().cpu().numpy() - rb[k]) / 0.1 / vb).max()
            e32 = np.abs((rb32[k] - rb[k]) / 0.1 / vb).max()
            vrow.append((eg, e32, k))
        vrow.sort(reverse=True)
        print("   batch var rel err (gpu / torch fp32):", ", ".join(f"{k.split('.')[0]}:{a:.1e}/{b:.1e}" for a, b, k in vrow[:5]))
        rows = []
        for pn, p in m.named_parameters():
            if O.bn_cancelled(pn):
                continue
            g = p.grad.double().cpu().numpy()
            r = rg[pn]
            nr = max(np.linalg.norm(r), 1e-30)
            e = np.linalg.norm(g - r) / nr
            fl = np.linalg.norm(r32[pn] - r) / nr
            rows.append((e / max(1e-2, 2 * fl), e, fl, pn))
        rows.sort(reverse=True)
        for q, e, fl, pn in rows[:6]:
            print(f"   {pn:50s} err {e:.3e} fp32-ref {fl:.3e} err/tol {q:.2f}")
        bn = [r for r in rows if O.is_bn_param(r[3])]
        print(f"   BN params: median err {np.median([r[1] for r in bn]):.2e} (fp32 ref {np.median([r[2] for r in bn]):.2e}),"
              f" worst err/tol {rows[0][0]:.2f}", flush=True)
        del m, logits, loss
        torch.cuda.empty_cache()
    for k, v in DEFAULTS.items():
        lib.unet_set_tuning(k.encode(), v)


if __name__ == "__main__":
    main()
