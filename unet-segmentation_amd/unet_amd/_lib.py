"""ctypes binding of libunet_hip.so (include/unet_hip.h).

This is the Python side of the C-ABI boundary.  The library is built in-tree
(``unet-segmentation_amd/csrc/Makefile`` -> ``unet_amd/libunet_hip.so``); there
is no fallback: if it cannot be loaded every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("UNET_HIP_LIB", os.path.join(_HERE, "libunet_hip.so"))

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t

# name -> (restype, argtypes); every symbol include/unet_hip.h declares.
SIGNATURES = {
    "unet_version": (ctypes.c_char_p, []),
    "unet_last_error": (ctypes.c_char_p, []),
    "unet_plan_create": (_vp, [_i, _i, _i, _i, _i]),
    "unet_plan_create_ex": (_vp, [_i, _i, _i, _i, _i, _i]),
    "unet_plan_precision": (_i, [_vp]),
    "unet_plan_destroy": (None, [_vp]),
    "unet_plan_out_hw": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "unet_plan_workspace_bytes": (_sz, [_vp]),
    "unet_plan_forward_workspace_bytes": (_sz, [_vp]),
    "unet_plan_num_params": (_i, [_vp]),
    "unet_plan_num_grads": (_i, [_vp]),
    "unet_plan_forward": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp]),
    "unet_plan_num_segments": (_i, [_vp]),
    "unet_plan_segment_grads": (_i, [_vp, _i, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "unet_plan_backward": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp]),
    "unet_plan_backward_ex": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp]),
    "unet_plan_wait_segment": (_i, [_vp, _i, _vp]),
    "unet_plan_input_grad_scratch_bytes": (_sz, [_vp]),
    "unet_plan_input_grad": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "unet_plan_join": (_i, [_vp, _vp]),
    "unet_plan_set_timing": (_i, [_vp, _i]),
    "unet_plan_timing": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "unet_plan_timing_mfma_flops": (_i, [_vp, _vp]),
    "unet_plan_timing_sites": (_sz, [_vp, ctypes.c_char_p, _sz]),
    "unet_wce_fwd_bwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp]),
    "unet_scale_by_device_scalar": (_i, [_vp, _sz, _vp, _vp]),
    "unet_scale_by_device_scalar_out": (_i, [_vp, _vp, _sz, _vp, _vp]),
    "unet_sgd_momentum": (_i, [_vp, _vp, _vp, _sz, _f, _f, _f, _i, _vp]),
    "unet_iou_counts": (_i, [_vp, _vp, _sz, _vp, _vp]),
    "unet_mask_from_logits": (_i, [_vp, _vp, _i, _i, _i, _vp]),
    "unet_tile_gather": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "unet_tile_scatter": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp]),
    "unet_instance_masks_ws_bytes": (_sz, [_i, _i, _i]),
    "unet_instance_masks": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    "unet_rand_index_ws_bytes": (_sz, [_i, _i]),
    "unet_rand_index": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp]),
    "unet_weight_map_ws_bytes": (_sz, [_i]),
    "unet_weight_map": (_i, [_vp, _i, _i, _i, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "unet_elastic_ws_bytes": (_sz, [_i, _i, _i]),
    "unet_elastic_deform": (_i, [_vp, _vp, _i, _i, _i, _vp, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp, _vp,
                                 _vp]),
    "unet_conv3x3_fwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "unet_conv3x3_dgrad": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp]),
    "unet_conv3x3_wgrad": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "unet_conv_ws_bytes": (_sz, [_i, _i, _i, _i, _i]),
    "unet_convT2_fwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp]),
    "unet_convT2_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "unet_maxpool2_fwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    "unet_maxpool2_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "unet_bn_train_fwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "unet_bn_train_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "unet_bn_ws_bytes": (_sz, [_i]),
    "unet_bn_relu_ws_bytes": (_sz, [_i, _i, _i, _i]),
    "unet_bn_relu_fwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _i, _vp, _vp, _vp, _vp,
                              _vp]),
    "unet_bn_relu_bwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "unet_conv_first_ws_bytes": (_sz, [_i, _i, _i, _i]),
    "unet_conv_first_fwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "unet_conv_first_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "unet_conv1x1_ws_bytes": (_sz, [_i]),
    "unet_conv1x1_fwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp]),
    "unet_conv1x1_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "unet_peak_probe": (_i, [_i, _i, ctypes.POINTER(ctypes.c_double), _vp]),
    "unet_tracker_create": (_vp, [_i, _i, ctypes.c_double, ctypes.c_double, _i]),
    "unet_tracker_destroy": (None, [_vp]),
    "unet_tracker_ws_bytes": (_sz, [_i, _i]),
    "unet_tracker_add_frame": (_i, [_vp, _vp, _i, _vp, _vp]),
    "unet_tracker_step_host": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "unet_tracker_num_tracks": (_i, [_vp]),
    "unet_tracker_tracks": (_i, [_vp, _vp, _i]),
    "unet_linear_sum_assignment": (_i, [ctypes.c_longlong, ctypes.c_longlong, _vp, _vp, _vp]),
    "unet_set_tuning": (_i, [ctypes.c_char_p, _i]),
    "unet_tuning_report": (_sz, [ctypes.c_char_p, _sz]),
    "unet_tuning_reset": (_i, []),
    "unet_slab_fallbacks": (ctypes.c_longlong, [_i]),
    "unet_nondeterministic_sites": (ctypes.c_longlong, [_i]),
    "unet_fused_bnb_sites": (ctypes.c_longlong, [_i]),
    "unet_tuning_save": (_i, [ctypes.c_char_p]),
    "unet_tuning_load": (_i, [ctypes.c_char_p]),
}

_lib = None
_load_error = None


def load():
    """Load the shared library (once).  Raises RuntimeError if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise RuntimeError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - exercised only without a build
        _load_error = (f"libunet_hip.so could not be loaded from {LIB_PATH} ({e}); "
                       "build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        raise RuntimeError(_load_error) from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().unet_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc}): {last_error()}")


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def ptr_array(tensors):
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def stream_of(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


# csrc/Makefile SRC_HASH: sha256 over these files, in this order
_HASHED = ["igemm.hip", "igemm_bf16.hip", "conv3_dma.hip", "conv3_ring.hip", "winograd.hip", "elementwise.hip", "elastic.hip",
           "tiling.hip", "weightmap.hip", "postproc.hip", "track.hip", "ops.hip", "plan.hip", "wgrad3_ring.hip",
           "conv3_ring_pt.hip", "peak.hip", "gemm_ring.hip", "wgradT_ring.hip", "conv3_flat.hip", "conv3_c64.hip", "unet_internal.h", "gemm_common.h", "ring_common.h", "conv3_ring_kernel.h",
           os.path.join("..", "..", "include", "unet_hip.h")]


def source_hash() -> str:
    """The hash csrc/Makefile compiles into unet_version(), recomputed from the
    sources in this tree (first 16 hex digits of sha256)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(_HERE, "..", "csrc")
    for f in _HASHED:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_identity() -> dict:
    """unet_version() of the loaded library, the hash of the tree's sources and
    whether the two agree (a stale .so shows up as src_match False)."""
    v = load().unet_version().decode()
    built = v.rsplit(" src ", 1)[-1].split()[0] if " src " in v else "unknown"
    tree = source_hash()
    return {"version": v, "lib_src": built, "tree_src": tree, "src_match": built == tree,
            "ablation_build": v.endswith(" ablations")}


def slab_fallbacks(reset: bool = False) -> int:
    """Slab-mode weight gradients that fell back to atomics (wslab too small)."""
    return int(load().unet_slab_fallbacks(1 if reset else 0))


def tuning_report() -> str:
    """The GEMM autotuner's choices (one line per GEMM shape)."""
    lib = load()
    n = lib.unet_tuning_report(None, 0)
    buf = ctypes.create_string_buffer(n)
    lib.unet_tuning_report(buf, n)
    return buf.value.decode()
