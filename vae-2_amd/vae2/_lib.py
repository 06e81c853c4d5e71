"""ctypes binding of libvae2_hip.so (the C ABI declared in include/vae2_hip.h).

The product path has exactly one compute backend: the HIP kernels in this
library.  Loading fails loudly when the library is missing; there is no CPU or
eager-PyTorch fallback.
"""
import ctypes
import os

import torch  # noqa: F401  (loads PyTorch's libamdhip64 first: one HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VAE2_LIB", os.path.join(_HERE, "libvae2_hip.so"))

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_vp = ctypes.c_void_p


class Act(ctypes.Structure):
    """vae2_act: NHWC view, element (n,y,x,c) at ptr[((n*h+y)*w+x)*ps + c]."""

    _fields_ = [("n", c_i64), ("h", c_i64), ("w", c_i64), ("c", c_i64), ("ps", c_i64)]


P_ACT = ctypes.POINTER(Act)


class BnLayer(ctypes.Structure):
    """vae2_bn_layer (include/vae2_hip.h): one layer of a multi-layer BN launch."""
    _fields_ = [("x", c_vp), ("xd", Act), ("a", c_vp), ("ad", Act), ("o", c_vp), ("od", Act),
                ("dy", c_vp), ("dyd", Act), ("dres", c_vp), ("dresd", Act),
                ("save", c_vp), ("gamma", c_vp), ("partials", c_vp), ("sums", c_vp),
                ("countp", c_vp), ("count", c_f64), ("relu", c_int), ("dres_acc", c_int),
                ("rx", c_vp), ("rxd", Act), ("rsave", c_vp), ("rgamma", c_vp),
                ("rpartials", c_vp), ("rsums", c_vp), ("rdx", c_vp), ("rdxd", Act),
                ("mask", c_vp)]


class BnFin(ctypes.Structure):
    """vae2_bn_fin (include/vae2_hip.h): one layer of a multi-layer BN reduction."""
    _fields_ = [("partials", c_vp), ("rows", c_i64), ("c", c_i64), ("sums", c_vp),
                ("countp", c_vp), ("count", c_f64), ("gamma", c_vp), ("beta", c_vp),
                ("running_mean", c_vp), ("running_var", c_vp), ("num_batches_tracked", c_vp),
                ("momentum", c_f32), ("eps", c_f32), ("save", c_vp), ("dgamma", c_vp),
                ("dbeta", c_vp)]

# name -> (restype, argtypes)
_SIGS = {
    "vae2_abi_version": (c_int, []),
    "vae2_last_error": (ctypes.c_char_p, []),
    "vae2_kernel_log": (c_int, [c_int]),
    "vae2_kernel_log_read": (c_i64, [ctypes.c_char_p, c_i64]),
    "vae2_conv2d_packed_size": (c_i64, [c_i64, c_i64, c_int, c_int]),
    "vae2_conv2d_pack_weight": (c_int, [c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp]),
    "vae2_conv2d_pack_weight_ld": (c_int, [c_vp, c_i64, c_i64, c_int, c_int, c_i64, c_vp, c_vp]),
    "vae2_conv2d_pack_weights": (c_int, [c_vp, c_i64, c_vp]),
    "vae2_conv2d_fwd_stats_rows": (c_i64, [c_vp, P_ACT, P_ACT, c_int, c_int, c_int]),
    "vae2_conv2d_set_mfma_bf16": (c_int, [c_int]),
    "vae2_conv2d_set_tune": (c_int, [c_int, c_int]),
    "vae2_wgrad_defer": (c_int, [c_int]),
    "vae2_wgrad_flush": (c_int, [c_vp]),
    "vae2_wgrad_flush_stream": (c_int, [c_vp]),
    "vae2_conv2d_set_algo": (c_int, [c_int]),
    "vae2_conv2d_fwd": (c_int, [c_vp, P_ACT, c_vp, c_vp, c_vp, P_ACT, c_int, c_int, c_int,
                                c_f32, c_vp, c_vp]),
    "vae2_conv2d_fwd_kernel_name": (c_int, [P_ACT, P_ACT, c_int, c_int, c_int, ctypes.c_char_p,
                                            c_i64]),
    "vae2_conv2d_bwd_data": (c_int, [c_vp, P_ACT, c_vp, c_vp, P_ACT, c_int, c_int, c_int,
                                     c_f32, c_vp]),
    "vae2_conv2d_bnin_ok": (c_int, [c_vp, P_ACT, P_ACT, c_int, c_int, c_int]),
    "vae2_conv2d_fwd_bnin": (c_int, [c_vp, P_ACT, c_vp, c_int, c_vp, c_vp, c_vp, P_ACT, c_int,
                                     c_int, c_int, c_f32, c_vp, c_vp]),
    "vae2_conv2d_bwd_weight_bnin": (c_int, [c_vp, P_ACT, c_vp, c_int, c_vp, P_ACT, c_vp, c_vp,
                                            c_int, c_int, c_int, c_int, c_vp, c_i64, c_vp]),
    "vae2_conv2d_bwd_data_bnpart_rows": (c_i64, [c_vp, P_ACT, P_ACT, c_int, c_int, c_int]),
    "vae2_conv2d_bwd_data_bnpart": (c_int, [c_vp, P_ACT, c_vp, c_vp, P_ACT, c_int, c_int, c_int,
                                            c_vp, P_ACT, c_vp, c_int, c_vp, c_vp]),
    "vae2_conv2d_bwd_weight_ws_size": (c_i64, [P_ACT, P_ACT, c_int]),
    "vae2_conv2d_bwd_weight": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, c_vp, c_int, c_int,
                                       c_int, c_int, c_vp, c_i64, c_vp]),
    "vae2_conv2d_bwd_weight_ld": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, c_i64, c_vp, c_int,
                                          c_int, c_int, c_int, c_vp, c_i64, c_vp]),
    "vae2_conv1x1_upsum_stats_rows": (c_i64, [P_ACT]),
    "vae2_conv1x1_upsum_fwd": (c_int, [c_vp, P_ACT, c_vp, c_vp, c_int, ctypes.POINTER(c_vp), P_ACT,
                                       c_vp, P_ACT, c_vp, c_vp]),
    "vae2_upsample_bilinear_bwd_multi_ws_size": (c_i64, [P_ACT, c_int, P_ACT]),
    "vae2_upsample_bilinear_bwd_multi": (c_int, [c_vp, P_ACT, c_int, ctypes.POINTER(c_vp), P_ACT,
                                                 c_vp, c_i64, c_vp]),
    "vae2_upsample_bilinear_bwd_pow2_ws_size": (c_i64, [P_ACT, c_int, P_ACT]),
    "vae2_upsample_bilinear_bwd_pow2": (c_int, [c_vp, P_ACT, c_int, ctypes.POINTER(c_vp), P_ACT,
                                                c_vp, c_vp, c_i64, c_vp]),
    "vae2_head_out_fwd":(c_int, [c_vp, P_ACT, c_vp, c_vp, c_vp, c_int, c_vp, P_ACT, c_vp]),
    "vae2_head_out_bwd_ws_size": (c_i64, [P_ACT, c_int]),
    "vae2_head_out_bwd_reduce": (c_int, [c_vp, P_ACT, c_vp, c_vp, c_int, c_vp, P_ACT, c_vp, c_vp,
                                         c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "vae2_head_out_bwd_apply": (c_int, [c_vp, P_ACT, c_vp, c_vp, c_vp, c_int, c_vp, P_ACT, c_vp,
                                        c_f64, c_vp, P_ACT, c_vp, c_vp, c_i64, c_vp]),
    "vae2_bn_reduce_finalize_shifted": (c_int, [c_vp, c_i64, c_i64, c_vp, c_f64, c_vp, c_vp, c_vp,
                                                c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp]),
    "vae2_bn_finalize_shifted": (c_int, [c_vp, c_f64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_f32, c_f32, c_i64, c_vp, c_vp]),
    "vae2_bn_partial_rows": (c_i64, [P_ACT]),
    "vae2_bn_stats": (c_int, [c_vp, P_ACT, c_vp, c_vp]),
    "vae2_bn_partials_reduce": (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_vp]),
    "vae2_bn_finalize": (c_int, [c_vp, c_f64, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32,
                                 c_i64, c_vp, c_vp]),
    "vae2_bn_reduce_finalize": (c_int, [c_vp, c_i64, c_i64, c_vp, c_f64, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_f32, c_f32, c_vp, c_vp]),
    "vae2_bn_bwd_reduce_param_grads": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "vae2_bn_eval_coeffs": (c_int, [c_vp, c_vp, c_vp, c_vp, c_f32, c_i64, c_vp, c_vp]),
    "vae2_bn_apply": (c_int, [c_vp, P_ACT, c_vp, c_vp, P_ACT, c_vp, P_ACT, c_int, c_vp]),
    "vae2_bn_relu_bwd_reduce": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, P_ACT, c_vp, c_int,
                                        c_vp, c_vp]),
    "vae2_bn_bwd_param_grads": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "vae2_bn_relu_bwd_apply": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, P_ACT, c_vp, c_vp,
                                       c_vp, c_f64, c_int, c_vp, P_ACT, c_vp, P_ACT, c_vp]),
    "vae2_upsample_bilinear_fwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_f32, c_vp]),
    "vae2_upsample_bilinear_bwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_f32, c_vp]),
    "vae2_fuse_sum_relu": (c_int, [c_int, ctypes.POINTER(c_vp), P_ACT, c_vp, P_ACT, c_vp]),
    "vae2_fuse_sum_relu_bn": (c_int, [c_int, ctypes.POINTER(c_vp), P_ACT, ctypes.POINTER(c_vp),
                                      c_vp, P_ACT, c_vp]),
    "vae2_relu_bwd_dual": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, P_ACT, c_vp, P_ACT, c_f32,
                                   c_vp]),
    "vae2_relu_bwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, P_ACT, c_vp]),
    "vae2_copy_act": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_f32, c_vp]),
    "vae2_codemap_tile_fwd": (c_int, [c_vp, c_i64, c_vp, P_ACT, c_vp]),
    "vae2_spatial_ws_size": (c_i64, [P_ACT]),
    "vae2_codemap_tile_bwd": (c_int, [c_vp, P_ACT, c_vp, c_i64, c_int, c_vp, c_i64, c_vp]),
    "vae2_nchw_to_nhwc": (c_int, [c_vp, c_vp, P_ACT, c_f32, c_vp]),
    "vae2_nhwc_to_nchw": (c_int, [c_vp, P_ACT, c_vp, c_f32, c_vp]),
    "vae2_global_avgpool_fwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, c_i64, c_vp]),
    "vae2_global_avgpool_bwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_f32, c_vp]),
    "vae2_reduce_ws_size": (c_i64, [c_i64]),
    "vae2_l1_fwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_f32, c_vp, c_vp, c_vp]),
    "vae2_l1_bwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, c_f32, c_vp, P_ACT, c_f32, c_vp]),
    "vae2_bn_multi_apply": (c_int, [c_int, c_vp, c_vp]),
    "vae2_bn_multi_bwd_reduce": (c_int, [c_int, c_vp, c_vp]),
    "vae2_bn_multi_bwd_apply": (c_int, [c_int, c_vp, c_vp]),
    "vae2_bn_multi_reduce": (c_int, [c_int, c_vp, c_int, c_vp]),
    "vae2_bn_multi_finalize": (c_int, [c_int, c_vp, c_vp]),
    "vae2_lsgan_fwd": (c_int, [c_vp, P_ACT, c_f32, c_f32, c_vp, c_vp, c_vp]),
    "vae2_lsgan_bwd": (c_int, [c_vp, P_ACT, c_f32, c_vp, c_f32, c_vp, P_ACT, c_f32, c_vp]),
    "vae2_reparam_kl_fwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, P_ACT, c_int, c_f32, c_vp,
                                    c_int, c_vp, c_vp]),
    "vae2_reparam_kl_bwd": (c_int, [c_vp, P_ACT, c_vp, P_ACT, c_vp, P_ACT, c_vp, c_f32, c_vp,
                                    P_ACT, c_vp]),
    "vae2_weighted_sum": (c_int, [c_int, ctypes.POINTER(c_vp), ctypes.POINTER(c_f32), c_vp,
                                  c_vp]),
    "vae2_nonfinite_check": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "vae2_adam_coeffs": (c_int, [c_vp, c_f32, c_f32, c_vp, c_vp]),
    "vae2_adam_step_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32, c_f32, c_f32,
                                   c_f32, c_vp]),
    "vae2_adam_step": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32,
                               c_i64, c_vp]),
    "vae2_scale": (c_int, [c_vp, c_vp, c_i64, c_f32, c_vp]),
    "vae2_syncbn_comm_bytes": (c_i64, [c_int, c_i64]),
    "vae2_syncbn_comm_init": (c_int, [c_int, c_int, c_i64, c_vp, ctypes.POINTER(c_vp)]),
    "vae2_syncbn_comm_connect": (c_int, [c_vp, c_vp]),
    "vae2_syncbn_allreduce": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "vae2_syncbn_comm_error": (c_int, [c_vp, ctypes.POINTER(c_i64)]),
    "vae2_syncbn_comm_set_timeout": (c_int, [c_vp, ctypes.c_double]),
    "vae2_syncbn_comm_destroy": (c_int, [c_vp]),
    "vae2_clip_normalize_u8": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_int,
                                       ctypes.POINTER(c_vp), c_vp]),
    "vae2_to_image": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64,
                              ctypes.POINTER(c_f64), ctypes.POINTER(c_f64), c_vp]),
    "vae2_metrics_ws_size": (c_i64, [c_i64, c_i64, c_i64]),
    "vae2_absdiff_sqdiff_sum": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "vae2_ssim": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_f32, c_f32, c_vp,
                          c_vp, c_vp]),
    "vae2_avgpool2x2": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "vae2_heads_set_algo": (c_int, [c_int]),
    "vae2_conv2d_multi": (c_int, [c_int, c_vp, c_vp]),
    "vae2_weighted_avgpool_fwd": (c_int, [c_vp, P_ACT, c_vp, c_vp, c_f32, c_vp, P_ACT, c_vp,
                                          c_i64, c_vp]),
    "vae2_weighted_avgpool_bwd": (c_int, [c_vp, P_ACT, c_vp, c_vp, c_f32, c_vp, P_ACT, c_f32,
                                          c_vp]),
    "vae2_conv2d_set_grouping": (c_int, [c_int]),
}

ABI_VERSION = 12
_lib = None


def load():
    """Load (once) and type the shared library; raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libvae2_hip.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no fallback compute path)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.vae2_abi_version() != ABI_VERSION:
        raise RuntimeError("libvae2_hip.so ABI version mismatch; rebuild it")
    _lib = lib
    return lib


def exported_symbols():
    return sorted(_SIGS)


class PackJob(ctypes.Structure):
    """vae2_pack_job (include/vae2_hip.h)."""
    _fields_ = [("w", c_vp), ("out", c_vp), ("cout", ctypes.c_int32), ("cin", ctypes.c_int32),
                ("k", ctypes.c_int32), ("mode", ctypes.c_int32), ("ld", ctypes.c_int32),
                ("pad_", ctypes.c_int32)]


class ConvJob(ctypes.Structure):
    """vae2_conv_job (include/vae2_hip.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("k", ctypes.c_int32), ("stride", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("x", c_vp), ("xd", Act), ("wp", c_vp), ("bias", c_vp),
                ("y", c_vp), ("yd", Act), ("beta", c_f32), ("stats", c_vp)]


class HipError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        msg = load().vae2_last_error()
        raise HipError(f"libvae2_hip error {rc}: {msg.decode() if msg else ''}")


CALL_HOOK = None  # vae2.prof.StepProfiler._call while a profiler is active


def call(name, *args):
    fn = getattr(load(), name)
    if CALL_HOOK is not None:
        check(CALL_HOOK(name, fn, args))
    else:
        check(fn(*args))
