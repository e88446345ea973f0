"""ctypes binding of the hipzap native library (``hipzap/_lib/libhipzap.so``).

The library is the in-tree build of ``hipzap/csrc`` (see :mod:`hipzap.build`). On a GPU host
every hipzap op goes through it; there is deliberately no silent eager-PyTorch fallback for
the hot ops — if the library is missing on a GPU host, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

# HIPZAP_DEBUG=1 selects the HZ_DEBUG variant (device-side contract checks, csrc/common.h HZ_DCHECK;
# build it with `python -m hipzap.build --debug`); failures are read with hipzap.utils.kcheck
DEBUG = os.environ.get("HIPZAP_DEBUG") == "1"
# plain os.path (no pathlib): this module is on the torch-free cold-start path, where pathlib's
# imports (urllib.parse, ipaddress, ...) are a few ms of the measured window
_LIB_PATH = os.path.join(os.path.dirname(os.path.realpath(__file__)), "_lib",
                         "libhipzap_debug.so" if DEBUG else "libhipzap.so")
if os.environ.get("HIPZAP_LIB"):  # same-box A/B of two builds (scripts/ab_lib.sh)
    _LIB_PATH = os.path.realpath(os.environ["HIPZAP_LIB"])
DEBUG_UNITS = ("conv", "gemm", "vision", "transformer", "lstm", "lmbatch", "pack", "block")
_lock = threading.Lock()
_lib = None

c_void_p, c_int, c_long, c_double = C.c_void_p, C.c_int, C.c_long, C.c_double
c_float_p = C.POINTER(C.c_float)


class ConvParams(C.Structure):
    _fields_ = [
        ("x", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("res", c_void_p), ("out", c_void_p),
        ("N", c_int), ("H", c_int), ("W", c_int), ("C", c_int),
        ("Cout", c_int), ("R", c_int), ("S", c_int), ("stride", c_int), ("pad", c_int), ("P", c_int), ("Q", c_int),
        ("M", c_int), ("K", c_int), ("ksteps", c_int),
        ("act", c_int), ("out_f32", c_int), ("out_rowmajor", c_int), ("ldo", c_int),
        ("x_rowmajor", c_int), ("ldx", c_int),
        ("tiles_n", c_int), ("kw", c_int),
        ("lnf", c_void_p),  # const HzLnFold* (device memory) or NULL
        ("x_f32", c_int), ("z_C", c_int), ("zinit", c_void_p), ("zbias", c_void_p), ("z_HW", c_int),
        ("pad_z", c_int),  # ResNet seams (block.hip seam_kernel)
    ]


class LnFold(C.Structure):
    """Mirror of HzLnFold (csrc/hipzap.h); copied to device memory, pointed to by ConvParams.lnf."""
    _fields_ = [("stats_in", c_void_p), ("c1", c_void_p), ("res_stats", c_void_p), ("res_gamma", c_void_p),
                ("res_beta", c_void_p), ("stats_out", c_void_p), ("nslab_in", c_int), ("nslab_res", c_int),
                ("ld_stats", c_int), ("inv_d", C.c_float), ("eps_in", C.c_float), ("eps_res", C.c_float)]


class PoolParams(C.Structure):
    _fields_ = [("x", c_void_p), ("out", c_void_p),
                ("N", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("P", c_int), ("Q", c_int),
                ("k", c_int), ("stride", c_int), ("pad", c_int)]


class LstmParams(C.Structure):
    _fields_ = [("w", c_void_p), ("bias", c_void_p), ("emb", c_void_p), ("lde", c_int), ("tok_seq", c_void_p),
                ("x_state", c_void_p), ("h_state", c_void_p), ("c_state", c_void_p), ("step", c_void_p),
                ("In", c_int), ("H", c_int), ("ldk", c_int), ("step_off", c_int), ("n_forced", c_void_p),
                ("bacc_val", c_void_p), ("bacc_idx", c_void_p), ("bmax_val", c_void_p), ("bmax_idx", c_void_p),
                ("nblk", c_int), ("V", c_int), ("pre", c_void_p), ("xtab", c_void_p), ("pre0", c_void_p),
                ("h0_state", c_void_p), ("c0_state", c_void_p), ("H0", c_int), ("pad0", c_int)]


class SamplerParams(C.Structure):
    _fields_ = [("keys", c_void_p), ("tok_seq", c_void_p), ("step", c_void_p), ("step_off", c_int), ("draws", c_void_p),
                ("n_forced", c_void_p), ("V", c_int), ("n_exclude", c_int), ("exclude", c_int * 8),
                ("bmax_val", c_void_p), ("bmax_idx", c_void_p), ("nblk", c_int), ("rpb", c_int),
                ("bacc_val", c_void_p), ("bacc_idx", c_void_p)]


class DecoderParams(C.Structure):
    _fields_ = [("w", c_void_p), ("bias", c_void_p), ("h_state", c_void_p), ("step", c_void_p),
                ("step_off", c_int), ("logits", c_void_p), ("V", c_int), ("H", c_int), ("ldk", c_int), ("keys", c_void_p),
                ("seed", c_void_p), ("bmax_val", c_void_p), ("bmax_idx", c_void_p), ("nblk", c_int),
                ("rpb", c_int), ("bacc_val", c_void_p), ("bacc_idx", c_void_p), ("n_exclude", c_int),
                ("exclude", c_int * 8), ("n_hh", c_int), ("hh_blocks", c_int), ("hh_w", c_void_p * 4),
                ("hh_b", c_void_p * 4), ("hh_h", c_void_p * 4), ("hh_out", c_void_p * 4), ("hh_H", c_int * 4),
                ("hh_ld", c_int * 4), ("hh_blk", c_int * 5)]

# batched AWD-LSTM decode (csrc/lmbatch.hip, csrc/lmserve.cpp)
class LmbCtl(C.Structure):
    _fields_ = [("tok", c_int), ("out", c_int), ("dec_t", c_int), ("rec", c_int)]


class LmbLayerParams(C.Structure):
    _fields_ = [("w", c_void_p), ("bias", c_void_p), ("h", c_void_p), ("x", c_void_p), ("c", c_void_p),
                ("gpar", c_void_p), ("ctl", c_void_p), ("H", c_int), ("Kh", c_int), ("Kx", c_int), ("R", c_int),
                ("Bp", c_int), ("step_off", c_int), ("emb", c_void_p), ("dbest", c_void_p), ("V", c_int),
                ("nb_act", c_int), ("outp", c_void_p), ("tok", c_void_p), ("embproj", c_void_p)]


class LmbEmbProjParams(C.Structure):
    _fields_ = [("w", c_void_p), ("emb", c_void_p), ("out", c_void_p), ("R", c_int), ("Kh", c_int), ("Kx", c_int),
                ("Vp", c_int)]


class LmbDecParams(C.Structure):
    _fields_ = [("w", c_void_p), ("bias", c_void_p), ("h", c_void_p), ("gpar", c_void_p), ("ctl", c_void_p),
                ("seed", c_void_p), ("dbest", c_void_p), ("logits", c_void_p), ("V", c_int), ("Vp", c_int),
                ("K", c_int), ("Bp", c_int), ("nblk", c_int), ("step_off", c_int), ("n_exclude", c_int),
                ("nb_act", c_int), ("exclude", c_int * 8)]


class LmbAdmitParams(C.Structure):
    _fields_ = [("block", c_void_p), ("ctl", c_void_p), ("seed", c_void_p), ("outp", c_void_p), ("gpar", c_void_p),
                ("Bp", c_int), ("U", c_int), ("n_layers", c_int), ("pad_", c_int), ("h", c_void_p * 4),
                ("c", c_void_p * 4), ("Kh", c_int * 4), ("H", c_int * 4)]


HZ_K_LMB_LAYER, HZ_K_LMB_DEC, HZ_K_LMB_ADMIT = 14, 15, 16
class PackConvParams(C.Structure):  # csrc/pack.hip (torch-free checkpoint cold start)
    _fields_ = [("w", c_void_p), ("gamma", c_void_p), ("beta", c_void_p), ("mean", c_void_p), ("var", c_void_p),
                ("bias_in", c_void_p), ("wf", c_void_p), ("bias_out", c_void_p), ("cout", c_int), ("cin", c_int),
                ("r", c_int), ("s", c_int), ("cin_p", c_int), ("rows", c_int), ("ksteps", c_int), ("pad_", c_int),
                ("eps", c_double)]

class FragPackParams(C.Structure):  # csrc/pack.hip hz_frag_pack_launch (batched AWD-LSTM packing)
    _fields_ = [("a", c_void_p), ("b", c_void_p), ("out", c_void_p), ("bias_a", c_void_p), ("bias_b", c_void_p),
                ("bias_out", c_void_p), ("R", c_int), ("K", c_int), ("nrows", c_int), ("interleave_h", c_int),
                ("ka", c_int), ("acols", c_int), ("lda", c_int), ("bcols", c_int), ("ldb", c_int), ("pad_", c_int)]


HH_ROWS = 16  # HZ_HH_ROWS (hipzap.h): rows per recurrent-partial workgroup of the decoder kernel


def _sig(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


def _load():
    lib = C.CDLL(_LIB_PATH, mode=C.RTLD_GLOBAL)
    P = c_void_p
    _sig(lib, "hz_conv_launch", c_int, C.POINTER(ConvParams), c_int, P)
    _sig(lib, "hz_conv2_launch", c_int, C.POINTER(ConvParams), C.POINTER(ConvParams), c_int, P)
    _sig(lib, "hz_maxpool_launch", c_int, C.POINTER(PoolParams), P)
    _sig(lib, "hz_avgpool_launch", c_int, P, P, c_int, c_int, c_int, c_int, P)
    _sig(lib, "hz_preprocess_launch", c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P)
    _sig(lib, "hz_cast_f32_bf16", c_int, P, P, c_long, P)
    _sig(lib, "hz_cast_bf16_f32", c_int, P, P, c_long, P)
    _sig(lib, "hz_prog_create", P)
    _sig(lib, "hz_prog_destroy", None, P)
    _sig(lib, "hz_prog_num_ops", c_int, P)
    _sig(lib, "hz_prog_add_conv", c_int, P, C.POINTER(ConvParams), c_int, c_int)
    _sig(lib, "hz_prog_add_conv2", c_int, P, C.POINTER(ConvParams), C.POINTER(ConvParams), c_int, c_int)
    _sig(lib, "hz_prog_add_maxpool", c_int, P, C.POINTER(PoolParams), c_int)
    _sig(lib, "hz_prog_add_avgpool", c_int, P, P, P, c_int, c_int, c_int, c_int, c_int)
    _sig(lib, "hz_prog_add_preprocess", c_int, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, c_int)
    _sig(lib, "hz_prog_add_memcpy", c_int, P, P, P, C.c_size_t, c_int)
    _sig(lib, "hz_prog_add_fork", c_int, P, c_int)
    _sig(lib, "hz_prog_add_join", c_int, P, c_int)
    _sig(lib, "hz_prog_run", c_int, P, P)
    _sig(lib, "hz_prog_capture", c_int, P, P)
    _sig(lib, "hz_prog_replay", c_int, P, P)
    _sig(lib, "hz_prog_is_captured", c_int, P)
    _sig(lib, "hz_prog_prepare", c_int, P)
    _sig(lib, "hz_prog_bench", c_double, C.POINTER(c_void_p), C.POINTER(c_void_p), c_int, c_int)
    _sig(lib, "hz_prog_bench2", c_int, C.POINTER(c_void_p), C.POINTER(c_void_p), c_int, c_int, c_int,
         C.POINTER(c_double))
    PP = C.POINTER(c_void_p)
    _sig(lib, "hz_serve_bench", c_int, PP, PP, PP, PP, C.c_uint64, PP, PP, C.c_uint64, c_int, c_int,
         C.POINTER(c_double), C.POINTER(c_double))
    _sig(lib, "hz_diag_launch", c_int, c_int, c_int, c_int, P, P, c_long, P)
    _sig(lib, "hz_prog_add_diag", c_int, P, c_int, c_int, c_int, P, P, c_long, c_int)
    _sig(lib, "hz_prog_replay_n", c_int, P, P, c_int)
    _sig(lib, "hz_launch_kernel", c_int, c_int, P, P)
    _sig(lib, "hz_experiments", c_int)
    _sig(lib, "hz_prog_add_kernel", c_int, P, c_int, P, C.c_size_t, c_int)
    _sig(lib, "hz_lstm_cell_launch", c_int, C.POINTER(LstmParams), P)
    _sig(lib, "hz_decoder_launch", c_int, C.POINTER(DecoderParams), P)
    _sig(lib, "hz_sampler_launch", c_int, C.POINTER(SamplerParams), P)
    _sig(lib, "hz_decoder_geometry", None, c_int, C.POINTER(c_int), C.POINTER(c_int))
    _sig(lib, "hz_prog_add_lstm", c_int, P, C.POINTER(LstmParams), c_int)
    _sig(lib, "hz_prog_add_decoder", c_int, P, C.POINTER(DecoderParams), c_int)
    _sig(lib, "hz_prog_add_sampler", c_int, P, C.POINTER(SamplerParams), c_int)
    _sig(lib, "hz_prog_add_step_bump", c_int, P, P, c_int, c_int)
    _sig(lib, "hz_step_bump_launch", c_int, P, c_int, P)
    # plan images (csrc/plan.cpp; hipzap/lite.py is the torch-free client)
    U64, D = C.c_uint64, c_double
    _sig(lib, "hz_abi_version", U64)
    _sig(lib, "hz_plan_last_error", C.c_char_p)
    _sig(lib, "hz_plan_open", P, C.c_char_p, c_int, c_int, C.POINTER(D))
    _sig(lib, "hz_plan_add_contexts", c_int, P, c_int, c_int)
    _sig(lib, "hz_plan_num_contexts", c_int, P)
    _sig(lib, "hz_plan_set_stream_priority", None, P, c_int)
    _sig(lib, "hz_plan_timings", None, P, C.POINTER(D))
    _sig(lib, "hz_plan_blob", P, P, C.POINTER(U64))
    _sig(lib, "hz_plan_host", P, P, c_int)
    _sig(lib, "hz_plan_device", P, P, c_int)
    _sig(lib, "hz_plan_stream", P, P, c_int)
    _sig(lib, "hz_plan_upload_stream", P, P)
    _sig(lib, "hz_plan_replay", c_int, P, c_int)
    _sig(lib, "hz_plan_sync", c_int, P, c_int)
    _sig(lib, "hz_plan_infer", c_int, P, c_int, P, U64, U64, P, U64, U64)
    _sig(lib, "hz_plan_bench", D, P, c_int)
    _sig(lib, "hz_plan_close", None, P)
    _sig(lib, "hz_plan_prog", P, P, c_int)
    _sig(lib, "hz_plan_capture_ctx", c_int, P, c_int)
    PP_ = C.POINTER(c_void_p)
    _sig(lib, "hz_exec_create", P, PP_, PP_, PP_, C.POINTER(U64), c_int, PP_, U64, c_int)
    _sig(lib, "hz_exec_create_batched", P, PP_, PP_, PP_, C.POINTER(U64), c_int, PP_, U64, c_int, c_int, D, c_int)
    _sig(lib, "hz_exec_batches", None, P, C.POINTER(U64))
    _sig(lib, "hz_exec_submit", c_int, P, PP_, P, C.POINTER(D))
    _sig(lib, "hz_exec_submit_rows", c_int, P, PP_, c_int, P, C.POINTER(D))
    _sig(lib, "hz_exec_stats", None, P, C.POINTER(U64), C.POINTER(U64))
    _sig(lib, "hz_exec_destroy", None, P)
    _sig(lib, "hz_exec_bench", c_int, P, c_int, c_int, PP_, C.POINTER(D), C.POINTER(D))
    _sig(lib, "hz_http_start", P, c_int, P)
    _sig(lib, "hz_http_set_fast", c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, C.c_char_p)
    _sig(lib, "hz_http_set_lm", c_int, P, P, c_int, c_int, c_int, c_int, C.c_char_p, U64, C.c_char_p)
    _sig(lib, "hz_http_respond", None, P, c_int, C.c_char_p, U64, C.c_char_p, U64)
    _sig(lib, "hz_http_stats", None, P, C.POINTER(U64))
    _sig(lib, "hz_http_stop", C.c_int, P)
    _sig(lib, "hz_pack_conv_launch", c_int, C.POINTER(PackConvParams), P)
    _sig(lib, "hz_frag_pack_launch", c_int, C.POINTER(FragPackParams), P)
    _sig(lib, "hz_upload_file", c_int, C.c_char_p, c_int, C.POINTER(U64), C.POINTER(U64), C.POINTER(c_void_p), P)
    _sig(lib, "hz_lmb_layer_launch", c_int, C.POINTER(LmbLayerParams), P)
    _sig(lib, "hz_lmb_dec_launch", c_int, C.POINTER(LmbDecParams), P)
    _sig(lib, "hz_lmb_admit_launch", c_int, C.POINTER(LmbAdmitParams), P)
    _sig(lib, "hz_lmb_dec_blocks", c_int, c_int)
    _sig(lib, "hz_lmb_create", P, P, c_int, P, P, c_int, c_int, c_int, c_int, P, P, c_int)
    _sig(lib, "hz_lmb_submit", c_int, P, P, c_int, c_int, C.c_uint64, P, P, C.POINTER(D))
    _sig(lib, "hz_lmb_stats", None, P, C.POINTER(U64))
    _sig(lib, "hz_lmb_set_lowload", c_int, P, P, c_int)
    _sig(lib, "hz_lmb_embproj_launch", c_int, P, P)
    _sig(lib, "hz_lmb_lo_replays", U64, P)
    _sig(lib, "hz_lmb_set_solo", c_int, P, P)
    _sig(lib, "hz_lmb_solo_replays", U64, P)
    _sig(lib, "hz_lmb_destroy", None, P)
    if DEBUG:
        for unit in DEBUG_UNITS:
            _sig(lib, f"hz_debug_poll_{unit}", c_int, C.POINTER(C.c_uint))
    for extra in _EXTRA_SIGS:
        extra(lib)
    return lib


# other modules register additional prototypes here before first load
_EXTRA_SIGS: list = []


def available() -> bool:
    return os.path.exists(_LIB_PATH)


def lib():
    """Return the loaded native library, building it first if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(_LIB_PATH):
                if os.environ.get("HIPZAP_NO_AUTOBUILD"):
                    raise RuntimeError(f"hipzap native library missing: {_LIB_PATH} (run python -m hipzap.build)")
                from . import build as _b
                _b.build(verbose=False, debug=DEBUG)
            _lib = _load()
    return _lib


def experiments() -> bool:
    """The loaded library carries the HZ_EXPERIMENTS kernels (M32 / LN-fold GEMM tiles, LM ring variants):
    ``python -m hipzap.build --experiments``, ``HIPZAP_LIB=.../libhipzap_exp.so``."""
    return bool(lib().hz_experiments())


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"hipzap native call {what} failed with code {rc}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


def stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
