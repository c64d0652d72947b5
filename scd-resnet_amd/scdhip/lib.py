"""ctypes binding of libscdhip.so (the C-ABI declared in include/scdhip.h).

This is the MI355X replacement for the reference's native-op bindings: the pybind11
``topPool/bottomPool/leftPool/rightPool`` modules (cornerPooling/source/topPool.cpp:76-85)
and the cuDNN/ATen kernels reached through torch.nn.  No torch C++ headers: device
pointers, sizes and the current HIP stream go through plain C.

The library is required: importing this module without it, or calling it with a CPU
tensor, raises -- there is no CPU or eager-PyTorch fallback on the product path.
"""
import ctypes
import os

import torch  # noqa: F401  (must be imported first: shares torch's libamdhip64.so.7)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCDHIP_LIB", os.path.join(HERE, "libscdhip.so"))

DT_F32 = 0
DT_BF16 = 1
DT_F16 = 2
MAX_TAPS = 16
MAX_PHASES = 4
STAT_REPLICAS = 64

c_int, c_long, c_float, c_double, c_size_t, c_void_p = (ctypes.c_int, ctypes.c_long, ctypes.c_float,
                                                        ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p)


class GemmPhase(ctypes.Structure):
    _fields_ = [("Qh", c_int), ("Qw", c_int), ("rho_h", c_int), ("rho_w", c_int), ("ntaps", c_int),
                ("dh", c_int * MAX_TAPS), ("dw", c_int * MAX_TAPS), ("wt", c_int * MAX_TAPS)]


class BnFinArgs(ctypes.Structure):
    """struct scd_bn_fin_args (include/scdhip.h): one layer of scd_bn_finalize_n."""
    _fields_ = [("stats", c_void_p), ("nrep", c_int), ("C", c_int), ("count", c_double), ("gamma", c_void_p),
                ("beta", c_void_p), ("running_mean", c_void_p), ("running_var", c_void_p), ("num_batches", c_void_p),
                ("momentum", c_float), ("eps", c_float), ("mean", c_void_p), ("invstd", c_void_p), ("scale", c_void_p),
                ("shift", c_void_p)]


class BnBwdFinArgs(ctypes.Structure):
    """struct scd_bn_bwd_fin_args (include/scdhip.h): one layer of scd_bn_bwd_finalize_n."""
    _fields_ = [("stats", c_void_p), ("nrep", c_int), ("C", c_int), ("count", c_double), ("gamma", c_void_p),
                ("mean", c_void_p), ("invstd", c_void_p), ("dgamma", c_void_p), ("dbeta", c_void_p),
                ("gscale", c_float), ("coef", c_void_p)]


class PackDesc(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("out", c_void_p), ("start", c_long), ("A", c_int), ("B", c_int), ("T", c_int),
                ("mode", c_int), ("ldp", c_int), ("row_off", c_int), ("a_off", c_int), ("a_tot", c_int)]


P = c_void_p
I = c_int
L = c_long
F = c_float
D = c_double
PP = ctypes.POINTER(c_void_p)
IP = ctypes.POINTER(c_int)
LP = ctypes.POINTER(c_long)

# name -> (restype, argtypes); mirrors include/scdhip.h one to one
SIGNATURES = {
    "scd_conv_gemm": (I, [I, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, ctypes.POINTER(GemmPhase), P]),
    "scd_conv_gemm_heads": (I, [I, P, P, P, P, I, I, I, I, I, IP, PP, PP, PP, P]),
    "scd_conv_gemm_heads_keep": (I, [I, P, P, P, P, I, I, I, I, I, IP, PP, PP, PP, P, I, P]),
    "scd_conv_gemm_bnbwd": (I, [I, P, P, P, I, I, I, I, I, I, I, I, I, I, I, ctypes.POINTER(GemmPhase), P, P, P, P,
                                P, P, P]),
    "scd_conv_wgrad_workspace": (c_size_t, [I, I, I, I]),
    "scd_conv_wgrad_nsplit": (I, [I, L, I, I, I]),
    "scd_conv_wgrad_nsplit2": (I, [I, L, I, I, I, I, I]),
    "scd_conv_wgrad": (I, [I, P, P, P, I, I, I, I, I, I, I, I, I, I, IP, IP, P]),
    "scd_wgrad_reduce": (I, [P, I, I, I, I, I, I, I, L, L, L, P, I, F, P]),
    "scd_wgrad_reduce_rows": (I, [P, I, I, I, I, I, IP, IP, LP, LP, LP, PP, I, I, F, P]),
    "scd_pack_weight": (I, [I, P, P, I, I, I, I, I, I, P]),
    "scd_pack_weights_batched": (I, [I, P, I, L, P]),
    "scd_pad_channels": (I, [I, P, L, I, I, P, P]),
    "scd_im2col_stem": (I, [I, P, P, I, I, I, I, I, I, I, I, I, I, P]),
    "scd_stem_conv_fwd": (I, [I, P, P, P, P, I, I, I, I, I, P]),
    "scd_stem_conv_wgrad_nsplit": (I, [L]),
    "scd_stem_conv_wgrad": (I, [I, P, P, P, P, P, I, I, I, I, I, I, P]),
    "scd_stem_bwd_nsplit": (I, []),
    "scd_conv_dgrad_s2": (I, [I, P, P, P, I, I, I, I, I, I, P]),
    "scd_stem_bwd_fused": (I, [I, P, P, P, P, P, P, P, P, P, P, I, P, I, I, I, I, I, P]),
    "scd_stem_bwd_combine": (I, [I, P, P, P, P, I, F, P]),
    "scd_stem_pool_bwd_bn": (I, [I, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, P]),
    "scd_stats_collapse": (I, [P, I, I, P]),
    "scd_stats_collapse_to": (I, [P, I, I, P, P]),
    "scd_bn_finalize": (I, [P, I, I, D, P, P, P, P, P, F, F, P, P, P, P, P]),
    "scd_bn_apply": (I, [I, P, P, I, L, P, P, P, P, P, I, P]),
    "scd_bn_bwd_reduce": (I, [I, P, P, P, P, P, P, P, I, L, P, P]),
    "scd_bn_bwd_finalize": (I, [P, I, I, D, P, P, P, P, P, F, P, P]),
    "scd_bn_finalize_n": (I, [ctypes.POINTER(BnFinArgs), I, P]),
    "scd_bn_bwd_finalize_n": (I, [ctypes.POINTER(BnBwdFinArgs), I, P]),
    "scd_bn_bwd_apply": (I, [I, P, P, P, P, P, P, I, L, P, P, P]),
    "scd_bn_bwd_reduce2": (I, [I, P, P, P, P, P, P, P, P, I, L, P, P, P]),
    "scd_bn_bwd_apply2": (I, [I, P, P, P, P, P, P, I, L, P, P, P]),
    "scd_stem_pool_fwd": (I, [I, P, P, P, P, P, I, I, I, I, I, I, P]),
    "scd_stem_pool_bwd": (I, [I, P, P, P, P, P, P, I, I, I, I, I, I, P]),
    "scd_heads_fwd": (I, [I, P, I, I, I, I, IP, PP, PP, PP, P]),
    "scd_heads_bwd_accsize": (c_size_t, [I, I, IP]),
    "scd_heads_bwd": (I, [I, P, I, I, I, I, IP, PP, PP, P, P, P]),
    "scd_heads_bwd_packed": (I, [I, P, I, I, I, I, IP, PP, PP, F, P, P, P, P]),
    "scd_heads_bwd_weight_finalize": (I, [P, I, I, IP, PP, PP, PP, I, F, P]),
    "scd_heads_bwd_packed_split": (I, [I, P, I, I, I, I, IP, I, PP, PP, F, P, P, P, P]),
    "scd_heads_sparse_bwd": (I, [I, P, P, I, I, I, I, I, I, IP, I, PP, PP, F, P, I, P, P, P, P, P, P]),
    "scd_heads_sparse_fixup": (I, [I, P, P, I, I, I, I, P, I, P, P, P, P, P, P, P, P, P]),
    "scd_focal_fwd": (I, [P, P, L, P, P, P]),
    "scd_l1_gather_fwd": (I, [P, I, I, I, P, P, P, I, I, I, P, P, P]),
    "scd_centernet_loss_finalize": (I, [P, I, P, I, P, P, P, P]),
    "scd_scale_by_device": (I, [P, L, P, I, P, P]),
    "scd_heads_keep_map": (I, [P, I, I, I, P, I, P, P]),
    "scd_centernet_loss_fwd": (I, [P, P, L, P, I, P, I, I, I, P, P, P, I, I, I, I, P, P, P, P, P, P, P, P]),
    "scd_centernet_loss_bwd_scale": (I, [P, L, I, I, P, I, P, I, P, I, P, P, P]),
    "scd_decode_workspace": (c_size_t, [I, I]),
    "scd_decode_topk": (I, [P, I, I, I, I, P, I, P, I, P, P, P, P, P, P, P, P]),
    "scd_augment_workspace": (c_size_t, [I]),
    "scd_augment_tiles": (I, [P, P, I, I, I, P, P, P, F, ctypes.c_ulonglong, P, P]),
    "scd_slide_workspace": (c_size_t, [I]),
    "scd_slide_tiles": (I, [P, I, I, I, I, I, I, I, I, I, I, P, P, P]),
    "scd_slide_detections": (I, [P, I, I, I, I, I, I, F, P, P, P, P]),
    "scd_ceval_count": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, F, P, P]),
    "scd_ceval_emit": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, F, P, PP, P]),
    "scd_ceval_summary_workspace": (c_size_t, [L]),
    "scd_ceval_summary": (I, [PP, ctypes.POINTER(c_long), L, P, I, P, P, P]),
    "scd_adam_step": (I, [P, P, P, P, L, F, F, F, F, F, F, F, P]),
    "scd_adam_step_dev": (I, [P, P, P, P, L, P, F, F, F, F, P, P]),
    "scd_sgd_step_dev": (I, [P, P, P, L, P, F, F, F, I, F, P, P]),
    "scd_render_center_targets": (I, [P, P, I, I, I, F, P, P, P, P, P]),
    "scd_cpool_fwd": (I, [I, I, P, P, P, I, I, I, I, P]),
    "scd_cpool_bwd": (I, [I, I, P, P, P, I, I, I, I, P]),
    "scd_nms": (I, [P, L, I, I, I, P, P]),
    "scd_topk": (I, [P, I, L, I, I, I, P, P, P, P, P, P]),
    "scd_focal_prob_fwd": (I, [P, P, L, P, P, P]),
    "scd_masked_l1_fwd": (I, [P, P, P, L, I, I, P, P, P]),
    "scd_peer_mailbox_bytes": (c_size_t, [I, I]),
    "scd_peer_alloc": (I, [c_size_t, PP]),
    "scd_peer_free": (I, [P]),
    "scd_peer_ipc_handle": (I, [P, P]),
    "scd_peer_ipc_open": (I, [P, PP]),
    "scd_peer_ipc_close": (I, [P]),
    "scd_peer_allreduce_f64": (I, [P, I, I, I, PP, I, ctypes.c_ulonglong, P, ctypes.c_uint, P]),
    "scd_event_create": (I, [PP]),
    "scd_event_destroy": (I, [P]),
    "scd_event_record": (I, [P, P]),
    "scd_event_elapsed_ms": (I, [P, P, ctypes.POINTER(c_float)]),
    "scd_calib_mfma_peak": (I, [P, I, I, P, P, P]),
    "scd_calib_set_stamps": (I, [P]),
    "scd_calib_stamped_build": (I, []),
    "scd_version": (ctypes.c_char_p, []),
}


class _Lib:
    def __init__(self, path):
        if not os.path.exists(path):
            raise RuntimeError("libscdhip.so not found at %s -- build it with `python -c 'import __graft_entry__ as g; "
                               "g.build()'` (make -C scd-resnet_amd/csrc).  There is no CPU fallback." % path)
        self.path = path
        self.dll = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(self.dll, name)
            fn.restype = res
            fn.argtypes = args
            setattr(self, name, fn)


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _Lib(LIB_PATH)
    return _LIB


def check(rc, name):
    if rc != 0:
        raise RuntimeError("libscdhip: %s failed with status %d%s" % (
            name, rc, " (invalid argument / unsupported shape)" if rc == 9001 else " (hipError)"))


def call(name, *args):
    rc = getattr(_LIB or lib(), name)(*args)
    if rc:
        check(rc, name)


def ptr_array(ptrs):
    arr = (c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def int_array(vals):
    arr = (c_int * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


def long_array(vals):
    arr = (c_long * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


def exported_symbols():
    return list(SIGNATURES)
