"""ctypes binding of libautovc_hip.so (the C-ABI declared in include/autovc_hip.h).

The library is loaded lazily, *after* ``import torch``, so the process has exactly one
HIP runtime (torch's libamdhip64.so.7 satisfies the .so's NEEDED entry).  There is no
fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import torch  # noqa: F401  (must precede the HIP library)

HERE = os.path.dirname(os.path.abspath(__file__))
# AVC_LIB_PATH: another build of the same ABI (same-box A/B timing of two builds, tools/ only)
LIB_PATH = os.environ.get("AVC_LIB_PATH") or os.path.join(HERE, "libautovc_hip.so")
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["gemm_ring.hip", "gemm_conv.hip", "gemm_nt.hip", "gemm_tt.hip", "gemm.hip", "bn.hip", "lstm.hip", "elem.hip", "norm.hip", "variants.hip", "melgan.hip", "fold.hip", "disc.hip", "events.hip"]
ABI_VERSION = 31

F32, BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_TANH, ACT_LEAKY, ACT_GELU, ACT_SIGMOID = 0, 1, 2, 3, 4, 5

c_void_p, c_int, c_ll, c_float, c_size = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_size_t


class Operand(ctypes.Structure):
    _fields_ = [("ptr", c_void_p), ("dtype", c_int), ("kstrided", c_int), ("ld", c_ll), ("batch_stride", c_ll),
                ("taps", c_int), ("pad", c_int), ("t_out", c_int), ("t_in", c_int), ("chans", c_int)]


class GemmDesc(ctypes.Structure):
    _fields_ = [("M", c_int), ("N", c_int), ("K", c_int), ("batch", c_int), ("a", Operand), ("b", Operand),
                ("c", c_void_p), ("ldc", c_ll), ("c_batch_stride", c_ll), ("bias", c_void_p),
                ("accumulate", c_int), ("split_k", c_int), ("bn_partial", c_void_p), ("compute", c_int),
                ("c_bf16", c_void_p), ("residual", c_void_p), ("cperm", c_int), ("row_bias", c_void_p),
                ("rb_t", c_int), ("rb_pad", c_int), ("c_bf16_act", c_int), ("act_grad_of", c_void_p),
                ("col_sum", c_void_p), ("col_sum_n", c_int), ("c_pre_bf16", c_void_p), ("act_grad_dtype", c_int),
                ("c_trans_rows", c_int)]


class BnFin(ctypes.Structure):
    _fields_ = [("gamma", c_void_p), ("beta", c_void_p), ("running_mean", c_void_p), ("running_var", c_void_p),
                ("num_batches_tracked", c_void_p), ("momentum", c_float), ("eps", c_float), ("nupd", c_int),
                ("mean", c_void_p), ("rstd", c_void_p), ("scale", c_void_p), ("shift", c_void_p),
                ("apply_bf16", c_void_p), ("apply_act", c_int)]


class BnbArgs(ctypes.Structure):
    _fields_ = [("y", c_void_p), ("y_dtype", c_int), ("mean", c_void_p), ("rstd", c_void_p), ("gamma", c_void_p),
                ("beta", c_void_p), ("act", c_int), ("coef", c_void_p), ("dgamma", c_void_p), ("dbeta", c_void_p),
                ("dbias", c_void_p), ("accumulate", c_int), ("ws", c_void_p), ("dy_bf16", c_void_p)]


class PackOp(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("src2", c_void_p), ("dst", c_void_p), ("kind", c_int), ("out_dtype", c_int),
                ("d0", c_int), ("d1", c_int), ("d2", c_int), ("pad_", c_int), ("ld_out", c_ll),
                ("ci0", c_int), ("cn", c_int), ("cpad", c_int), ("mode", c_int)]


PACK_COPY, PACK_TRANSPOSE, PACK_CONV_F, PACK_CONV_D, PACK_ADD, PACK_CONV_SLICE = 0, 1, 2, 3, 4, 5


_SIGS = {
    "avc_abi_version": (c_int, []),
    "avc_last_error": (ctypes.c_char_p, []),
    "avc_ring_reserve_test": (ctypes.c_uint, [ctypes.POINTER(ctypes.c_uint), ctypes.c_uint, ctypes.c_uint]),
    "avc_gemm": (c_int, [ctypes.POINTER(GemmDesc), c_void_p]),
    "avc_expand_codes": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_code_cat": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_gemm_bn": (c_int, [ctypes.POINTER(GemmDesc), ctypes.POINTER(BnFin), c_void_p]),
    "avc_bn_finalize": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                                c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "avc_bn_eval": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p]),
    "avc_bn_stats": (c_int, [c_void_p, c_ll, c_int, c_int, c_void_p, c_void_p]),
    "avc_bn_apply": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                              c_void_p]),
    "avc_gemm_bnb_ws": (c_size, [c_int, c_int]),
    "avc_gemm_bnb": (c_int, [ctypes.POINTER(GemmDesc), ctypes.POINTER(BnbArgs), c_void_p]),
    "avc_bn_bwd_apply": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p]),
    "avc_bn_bwd_ws": (c_size, [c_int, c_int]),
    "avc_bn_bwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                           c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                           c_void_p]),
    "avc_colsum_ws": (c_size, [c_int, c_int]),
    "avc_colsum": (c_int, [c_void_p, c_ll, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "avc_lstm_fwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_int, c_void_p]),
    "avc_lstm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                             c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "avc_lstm_fwd_fold": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p]),
    "avc_lstm_bwd_fold": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "avc_lstm_bwd_scratch_bytes": (c_size, [c_int, c_int, c_int]),
    "avc_lstm2_persistent": (c_int, [c_int, c_int, c_int, c_int]),
    "avc_lstm2_scratch_bytes": (c_size, [c_int, c_int]),
    "avc_lstm2_fwd": (c_int, [c_void_p] * 5 + [c_int] * 3 + [c_void_p] * 10),
    "avc_lstm_trace": (c_int, [c_void_p]),
    "avc_set_fault_word": (c_int, [c_void_p]),
    "avc_lstm_set_spin": (c_int, [ctypes.c_uint]),
    "avc_gemm_set_ring": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "avc_gemm_ring_last": (c_int, []),
    "avc_lstm2_bwd_persistent": (c_int, [c_int, c_int, c_int]),
    "avc_lstm2_bwd_scratch_bytes": (c_size, [c_int, c_int]),
    "avc_lstm2_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                              c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "avc_lstm_persistent": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "avc_lstm_small_mfma": (c_int, [c_int, c_int]),
    "avc_lstm_set_small_mfma": (c_int, [c_int]),
    "avc_enc_concat": (c_int, [c_void_p, c_ll, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_codes_gather": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_codes_scatter": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_dec_concat": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_dec_concat_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_conv_pack": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_conv_grad_unpack": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_event_create": (c_int, [c_void_p]),
    "avc_event_record": (c_int, [c_void_p, c_void_p]),
    "avc_stream_wait_event": (c_int, [c_void_p, c_void_p]),
    "avc_conv_pack_slice": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_void_p]),
    "avc_conv_edge_table": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "avc_conv_edge_colsum": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "avc_conv_grad_unpack_slice": (c_int, [c_void_p, c_ll, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                           c_void_p]),
    "avc_disc_dense_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "avc_disc_dense_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "avc_convert": (c_int, [c_void_p, c_void_p, c_int, c_ll, c_void_p]),
    "avc_transpose": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_ll, c_void_p]),
    "avc_add": (c_int, [c_void_p, c_void_p, c_void_p, c_ll, c_void_p]),
    "avc_mse_loss": (c_int, [c_void_p, c_void_p, c_ll, c_void_p, c_void_p]),
    "avc_l1_loss": (c_int, [c_void_p, c_void_p, c_ll, c_void_p, c_void_p]),
    "avc_loss_grad": (c_int, [c_void_p, c_void_p, c_ll, c_void_p, c_int, c_void_p, c_float, c_void_p]),
    "avc_vc_loss_ws": (c_size, []),
    "avc_vc_loss": (c_int, [c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_ll, c_float, c_void_p, c_void_p,
                            c_void_p]),
    "avc_vc_loss_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_ll, c_float, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "avc_pack_batch": (c_int, [c_void_p, c_void_p, c_int, c_ll, c_void_p]),
    "avc_adam_blocks": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_float, c_float, c_float, c_float,
                                c_void_p, c_int, c_int, c_void_p]),
    "avc_adam": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_float, c_float, c_float, c_float, c_void_p,
                         c_int, c_void_p]),
    "avc_act_fwd": (c_int, [c_void_p, c_void_p, c_ll, c_int, c_void_p]),
    "avc_act_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p]),
    "avc_bce_loss": (c_int, [c_void_p, c_ll, c_float, c_void_p, c_void_p]),
    "avc_bce_grad": (c_int, [c_void_p, c_ll, c_float, c_void_p, c_void_p, c_int, c_void_p]),
    "avc_norm_ws": (c_size, [c_int, c_int]),
    "avc_group_norm_fwd": (c_int, [c_void_p, c_int, c_ll, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "avc_group_norm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_ll, c_int, c_void_p,
                                   c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "avc_layer_norm_fwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "avc_layer_norm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                   c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "avc_group_norm_fwd2": (c_int, [c_void_p, c_int, c_ll, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p]),
    "avc_layer_norm_fwd2": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    "avc_layer_norm_bwd2": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "avc_gelu_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_ll, c_void_p]),
    "avc_pool3_mixer": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_patchify": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_patchify16": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_transpose_batched": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_transpose_batched2": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                       c_void_p]),
    "avc_moments_ws": (c_size, []),
    "avc_moments": (c_int, [c_void_p, c_ll, c_void_p, c_void_p, c_void_p]),
    "avc_moments_bwd": (c_int, [c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "avc_adain_fwd": (c_int, [c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "avc_adain_bwd": (c_int, [c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p]),
    "avc_segsum": (c_int, [c_void_p, c_ll, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "avc_mg_gather": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                              c_void_p, c_int, c_void_p]),
    "avc_mg_act": (c_int, [c_void_p, c_ll, c_float, c_void_p, c_void_p, c_void_p]),
    "avc_mg_wn_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                               c_int, c_void_p, c_void_p]),
    "avc_mg_conv_out": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p,
                                c_void_p]),
    "avc_step_select": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_rownorm_fwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "avc_rownorm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "avc_crop_add": (c_int, [c_void_p, c_ll, c_void_p, c_int, c_int, c_void_p]),
    "avc_pad_cols": (c_int, [c_void_p, c_ll, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "avc_gelu_twin": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p]),
}

_lib = None
_lock = threading.Lock()


def build(verbose: bool = False, force: bool = False) -> str:
    """Compile csrc/*.hip for gfx950 into libautovc_hip.so (in-tree)."""
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    if not force and os.path.exists(LIB_PATH):
        import glob

        # every header a translation unit includes (csrc/*.h, the public ABI header)
        deps = srcs + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(HERE, "..", "include", "autovc_hip.h")]
        newest = max(os.path.getmtime(p) for p in deps)
        if os.path.getmtime(LIB_PATH) >= newest:
            return LIB_PATH
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = LIB_PATH + ".tmp"
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-pass-failed"]
    objdir = os.path.join(HERE, "_build")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(p) + ".o") for p in srcs]
    # one hipcc per translation unit, concurrently (the gfx950 device compile dominates)
    procs = []
    for src, obj in zip(srcs, objs):
        cmd = [hipcc] + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd, cwd=CSRC)))
    failed = [cmd for cmd, pr in procs if pr.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs, check=True, cwd=CSRC)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libautovc_hip.so not found at {LIB_PATH}; run autoformer_amd._lib.build() "
                               "(or __graft_entry__.build()). There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        v = L.avc_abi_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"libautovc_hip ABI {v} != expected {ABI_VERSION}; rebuild")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().avc_last_error().decode(errors="replace")
        raise RuntimeError(f"libautovc_hip {what} failed ({rc}): {msg}")


_FNS = {}  # name -> bound ctypes function (one dict lookup per launch instead of lib() + getattr)


_REC = None  # a replay.StepRecord while a step is being recorded (replay.recording)


def call(name: str, *args) -> None:
    fn = _FNS.get(name)
    if fn is None:
        fn = _FNS[name] = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        check(rc, name)
    if _REC is not None:
        _REC.add_native(fn, name, args)


def exported_symbols():
    return list(_SIGS.keys())
