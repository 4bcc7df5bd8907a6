"""CPU checks of the oracle's bf16-GEMM restatement (UNetOracle(gemm="bf16")),
the reference the HIP UNET_PREC_BF16 path is compared with."""
import numpy as np
import torch

from oracle import unet_oracle as O
from oracle import fixtures as F


def test_round_bf16_matches_torch_cast():
    rng = np.random.default_rng(0)
    x = np.concatenate([
        rng.standard_normal(50000) * 3,
        rng.standard_normal(5000) * 1e-30,  # subnormal range of bf16's fp32 exponent
        # exact ties: 1 + k/256 + 1/512 sits halfway between two bf16 values
        1.0 + np.arange(64) / 128.0 + 1.0 / 256.0,
        [0.0, -0.0, 1.0, -2.5, 65504.0, 3.4e38],
    ]).astype(np.float32)
    ref = torch.from_numpy(x).to(torch.bfloat16).float().double().numpy()
    np.testing.assert_array_equal(O.round_bf16(x), ref)


def test_bf16_oracle_is_a_perturbation_of_the_fp64_path():
    """bf16 operands move the logits by well under bf16 epsilon x depth.  (Deep
    weight gradients at this tiny size are not compared: their BatchNorm layers
    see 16-64 samples per channel and amplify any perturbation -- 30 % for up1
    and even inc.c0 at 188 px -- which is the network's sensitivity, not the rounding's.)"""
    params = O.hash_init(1, 2, seed=3, bn_random=True)
    x, t, w = F.make_inputs(3, 1, 1, 188)
    l64, c64, _ = O.UNetOracle(params).forward(x)
    lbf, cbf, _ = O.UNetOracle(params, gemm="bf16").forward(x)
    rel = np.linalg.norm(lbf - l64) / np.linalg.norm(l64)
    assert 1e-5 < rel < 5e-2
    g64 = O.UNetOracle(params).backward(O.weighted_ce(l64, t, w)[1], c64)
    gbf = O.UNetOracle(params, gemm="bf16").backward(O.weighted_ce(lbf, t, w)[1], cbf)
    for k in ("outc.conv.weight", "up4.conv.double_conv.3.weight"):
        e = np.linalg.norm(gbf[k] - g64[k]) / np.linalg.norm(g64[k])
        assert e < 0.1, (k, e)
