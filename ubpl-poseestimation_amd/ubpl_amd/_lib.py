"""Bindings of libubpl_hip.so (C-ABI declared in include/ubpl_hip.h).

Compute entry points are called through their torch ops — libubpl_ops.so,
TORCH_LIBRARY(ubpl, m), generated from the header by csrc/gen_torch_ops.py:
`ubpl::<name>` per C entry, device pointers as tensors, enqueued on torch's
current HIP stream.  The host-only planning queries (workspace sizes, plan
choices) and the ABI checks of the CPU tests use ctypes on the C-ABI itself.

torch is imported first so that both libraries bind to the HIP runtime torch
already loaded (same SONAME, one runtime, one set of streams).  There is no
CPU fallback: a missing library or a missing GPU raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# UBPL_LIB_DIR: another build of the same two libraries (same-box A/B of a kernel change)
_LIB_DIR = os.environ.get("UBPL_LIB_DIR") or _HERE
LIB_PATH = os.path.join(_LIB_DIR, "libubpl_hip.so")
OPS_PATH = os.path.join(_LIB_DIR, "libubpl_ops.so")

P, I, L, F, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double

# name -> (restype, argtypes) — mirrors include/ubpl_hip.h
SIGNATURES = {
    "ubpl_render_heatmaps": (I, [P, P, P, I, I, I, I, I, I, F, F, F, P]),
    "ubpl_heatmap_row_stats": (I, [P, L, L, P, L, L, L, I, I, I, I, I, P, P, P, P]),
    "ubpl_loss_finalize": (I, [I, P, P, P, P, P, I, I, I, I, I, F, P, P, P, P, P]),
    "ubpl_heatmap_row_grad": (I, [P, L, L, P, L, L, L, I, I, I, I, I, P, P, F, P, I, P]),
    "ubpl_fdl_cov_forward": (I, [P, P, P, I, I, I, I, P, P, P, P, P, P]),
    "ubpl_fdl_cov_backward": (I, [P, P, P, P, P, P, P, P, I, I, I, I, P, P, I, P]),
    "ubpl_decode_heatmaps": (I, [P, I, I, I, I, P, P, P, P, P]),
    "ubpl_pck": (I, [P, P, I, I, I, I, F, P, P, P, P, P]),
    "ubpl_ema_update": (I, [P, P, L, D, P]),
    "ubpl_adamw_step": (I, [P, P, P, P, L, D, D, D, D, D, L, P]),
    "ubpl_adamw_step_dev": (I, [P, P, P, P, L, D, D, D, D, D, P, P, P]),
    "ubpl_adamw_ema_step_dev": (I, [P, P, P, P, L, D, D, D, D, D, P, P, P, L, D, P]),
    "ubpl_scale_": (I, [P, L, F, P]),
    "ubpl_bn_splits": (I, [I, I]),
    "ubpl_bn_part_doubles": (L, [I, I]),
    "ubpl_bn_forward_stats": (I, [P, I, I, I, P, P, F, F, P, P, P, P, P, P, P, P]),
    "ubpl_bn_eval_coeffs": (I, [P, P, P, P, F, I, P, P, P]),
    "ubpl_bn_apply": (I, [P, I, I, I, P, P, I, P, P]),
    "ubpl_bn_partial_floats": (L, [I, L]),
    "ubpl_bn_partials": (I, [P, I, I, I, P, P]),
    "ubpl_bn_stats_from_partials": (I, [P, I, L, P, P, F, F, P, P, P, P, P, P, P]),
    "ubpl_bn_backward_split": (I, [P, P, I, I, I, I, P, P, P, P, P, I, P, P, P, P, P, I, I, P, L, P]),
    "ubpl_bn_backward": (I, [P, P, I, I, I, P, P, P, P, P, I, P, P, P, P, P, P, P, P, P]),
    "ubpl_bn_backward_partials": (I, [P, P, I, I, I, P, P, P, I, P, P]),
    "ubpl_conv2d_forward": (I, [P, I, I, I, I, P, P, I, I, I, P, P, P, P, I, I, P, P]),
    "ubpl_conv2d_forward_workspace": (L, [I, I, I, I, I, I]),
    "ubpl_conv1x1_kmajor_workspace": (L, [I, I, I, I]),
    "ubpl_conv1x1_forward_kmajor": (I, [P, I, I, I, P, P, I, P, P, P, P, P, P, P]),
    "ubpl_conv_weight_tapmajor": (I, [P, I, I, I, P, P]),
    "ubpl_conv2d_wgrad_workspace": (L, [I, I, I, I, I, I]),
    "ubpl_conv2d_wgrad": (I, [P, P, I, I, I, I, I, I, I, P, P, I, I, P, P, P, I, P]),
    "ubpl_conv_weight_flip": (I, [P, I, I, I, P, P]),
    "ubpl_conv_weights_relayout": (I, [P, P, P, I, I, P]),
    "ubpl_wgrad_slab_reduce": (I, [P, I, I, I, I, I, P, P, I, P]),
    "ubpl_wgrad3_psa_workspace": (L, [I, I, I, I, I]),
    "ubpl_wgrad3_psa": (I, [P, L, P, L, I, I, I, I, I, P, P, P, I, I, P, P]),
    "ubpl_wgrad_stem_psa_workspace": (L, [I, I, I, I]),
    "ubpl_wgrad_stem_psa": (I, [P, L, P, L, I, I, I, I, I, I, P, P, P, I, I, P]),
    "ubpl_wgrad1x1_split_load_workspace": (L, [I, I, I, I]),
    "ubpl_wgrad1x1_split_load": (I, [P, P, I, I, I, I, P, P, P, P, P, I, I, P]),
    "ubpl_conv2d_forward_split_workspace": (L, [I, I, I, I, I, I, I]),
    "ubpl_conv2d_forward_split": (I, [P, I, I, I, I, P, L, P, I, I, I, P, P, P, P, I, I, P, I, P]),
    "ubpl_conv_weights_split": (I, [P, P, L, P, I, I, I, P]),
    "ubpl_split_activation": (I, [P, I, I, I, I, P, P, I, I, P, L, P, L, P]),
    "ubpl_conv2d_forward_psa_workspace": (L, [I, I, I, I, I, I, I]),
    "ubpl_set_psa_dispatch": (I, [I, I]),
    "ubpl_conv2d_forward_psa": (I, [P, L, I, I, I, I, I, P, L, P, I, I, P, P, P, I, P, P, P, I, P, P, P]),
    "ubpl_stem_s2d_split": (I, [P, I, I, I, I, I, I, P, L, P]),
    "ubpl_stem_weight_s2d_split": (I, [P, I, I, I, I, P, L, P]),
    "ubpl_conv1x1_split_load_preferred": (I, [I, I, I, I]),
    "ubpl_conv1x1_forward_split_load": (I, [P, I, I, I, P, L, P, I, P, P, P, P, P, P, P, I, P, I, P]),
    "ubpl_maxpool2x2_forward": (I, [P, L, I, I, P, P]),
    "ubpl_maxpool2x2_backward": (I, [P, P, L, I, I, P, I, P]),
    "ubpl_avgpool2x2_forward": (I, [P, L, I, I, P, P]),
    "ubpl_avgpool2x2_backward": (I, [P, L, I, I, P, I, P]),
    "ubpl_upsample2x_add_forward": (I, [P, P, L, I, I, P, P]),
    "ubpl_maxpool2x2_forward_stats": (I, [P, I, I, I, I, P, P, P]),
    "ubpl_upsample2x_add_forward_stats": (I, [P, P, I, I, I, I, P, P, P]),
    "ubpl_upsample2x_add_backward": (I, [P, L, I, I, P, I, P]),
    "ubpl_add": (I, [P, P, L, P, P]),
    "ubpl_image_mean_u8": (I, [P, I, L, P, P]),
    "ubpl_augment_warp": (I, [P, I, I, P, P, P, P, P, I, I, I, P, P]),
    "ubpl_occlude": (I, [P, I, I, I, P, P, P, P, P, P, P]),
    "ubpl_augment_chain": (I, [P, I, I, P, P, P, P, P, I, I, I, P, I, I, P, P]),
}

_lib = None


def load(path=LIB_PATH):
    """Load the library and bind every symbol (raises if any is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError("ubpl_amd: %s not found — build it with `make -C ubpl-poseestimation_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback" % path)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load()


def require_gpu(t=None):
    if not torch.cuda.is_available():
        raise RuntimeError("ubpl_amd: the HIP hot path needs an MI355X (gfx950) GPU; no CPU fallback")
    if t is not None and not t.is_cuda:
        raise RuntimeError("ubpl_amd: expected a device tensor, got %s" % t.device)


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def check(rc, name):
    if rc != 0:
        raise RuntimeError("ubpl_amd: %s failed with hipError %d" % (name, rc))


_ops = {}


def load_ops(path=OPS_PATH):
    """Register the ubpl torch ops (raises if the library is missing)."""
    if not _ops:
        lib()
        if not os.path.exists(path):
            raise RuntimeError("ubpl_amd: %s not found — build it with `make -C ubpl-poseestimation_amd/csrc` "
                               "(or __graft_entry__.build()); there is no CPU fallback" % path)
        torch.ops.load_library(path)
        _ops["loaded"] = True
    return torch.ops.ubpl


def op(name):
    """The torch op (OpOverload) of C-ABI entry `name`."""
    o = _ops.get(name)
    if o is None:
        o = _ops[name] = getattr(load_ops(), name[len("ubpl_"):]).default
    return o


def call(name, *args):
    """Enqueue C-ABI entry `name` through its torch op.  `args` follow the C
    signature (device pointers as tensors or None) without its trailing
    stream argument: the op enqueues on torch's current stream."""
    return op(name)(*args)
