"""ctypes binding of libgpmdm_hip.so (declarations: include/gpmdm_hip.h).

The library is the product path: nothing here falls back to a CPU implementation.  If
the shared object is missing, ``load()`` raises with the build command; if a call fails,
the library's status is mapped to ``ValueError`` (bad argument, as the reference raises)
or ``RuntimeError`` (HIP failure / out-of-order call).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint64, c_void_p
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libgpmdm_hip.so"

GPMDM_OK = 0
GPMDM_E_INVALID = -1
GPMDM_E_HIP = -2
GPMDM_E_NOMEM = -3
GPMDM_E_STATE = -4
GPMDM_RNG_REPLAY = 0
GPMDM_RNG_PHILOX = 1
GPMDM_RESAMPLE_MULTINOMIAL = 0
GPMDM_RESAMPLE_SYSTEMATIC = 1
GPMDM_PACK_ALL, GPMDM_PACK_STATES, GPMDM_PACK_LL = 0, 1, 2
GPMDM_COMM_PAD_ROWS = 1
GPMDM_COMM_ID_BYTES = 128
DYN_TILES = {"auto": 0, "narrow": 1, "wide": 2}
STAGES = ("switch", "dyn_gemm", "dyn_finish", "obs_gemm", "obs_finish", "resample")
HEALTH = ("obs_var_nonpositive", "obs_ll_nonfinite", "dyn_var_nonpositive", "dyn_state_nonfinite")

_dp = POINTER(c_double)
_i64p = POINTER(c_int64)


class ModelDesc(ctypes.Structure):
    _fields_ = [
        ("N", c_int64), ("D", c_int32), ("d", c_int32), ("C", c_int32), ("tile_shape", c_int32),
        ("X", _dp), ("obs_R", _dp), ("obs_beta", _dp),
        ("y_lengthscales", _dp), ("y_inv_lambda2", _dp),
        ("Nc", _i64p), ("Xin", POINTER(_dp)), ("dyn_R", POINTER(_dp)), ("dyn_alpha", POINTER(_dp)),
        ("x_lengthscales", _dp), ("x_lin_coeff2", _dp), ("x_inv_lambda2", _dp),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "gpmdm_model_create": (c_int, [POINTER(ModelDesc), c_int, POINTER(c_void_p)]),
    "gpmdm_model_destroy": (c_int, [c_void_p]),
    "gpmdm_predict_obs": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "gpmdm_predict_dyn": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "gpmdm_pf_create": (c_int, [c_void_p, _dp, c_int64, c_int, c_uint64, c_int, c_int, c_int, POINTER(c_void_p)]),
    "gpmdm_pf_destroy": (c_int, [c_void_p]),
    "gpmdm_bank_create": (c_int, [c_void_p, _dp, c_int64, c_int64, c_uint64, c_int, POINTER(c_void_p)]),
    "gpmdm_pf_shape": (c_int, [c_void_p, _i64p, _i64p]),
    "gpmdm_pf_init": (c_int, [c_void_p, _dp, _i64p]),
    "gpmdm_pf_import": (c_int, [c_void_p, _dp, _i64p, _dp, _dp, _dp, _i64p, c_int64]),
    "gpmdm_pf_draw_buffers": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p)]),
    "gpmdm_pf_draws_free": (c_int, [c_void_p, c_int]),
    "gpmdm_pf_switch": (c_int, [c_void_p, _dp, _i64p, c_void_p]),
    "gpmdm_pf_preswitch": (c_int, [c_void_p, _dp, c_void_p]),
    "gpmdm_pf_stage_normals": (c_int, [c_void_p, _dp, c_int64, c_int64, c_void_p]),
    "gpmdm_pf_propagate": (c_int, [c_void_p, _dp, _dp, c_void_p]),
    "gpmdm_pf_propagate_dynamics": (c_int, [c_void_p, _dp, c_void_p]),
    "gpmdm_pf_weigh": (c_int, [c_void_p, _dp, c_void_p]),
    "gpmdm_pf_exchange_width": (c_int, [c_void_p, _i64p, _i64p, _i64p]),
    "gpmdm_pf_pack": (c_int, [c_void_p, c_void_p, c_void_p]),
    "gpmdm_pf_unpack": (c_int, [c_void_p, c_void_p, c_void_p]),
    "gpmdm_pf_pack_part": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "gpmdm_pf_unpack_part": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "gpmdm_pf_resample": (c_int, [c_void_p, _dp, c_void_p]),
    "gpmdm_pf_step": (c_int, [c_void_p, _dp, _dp, _dp, _dp, c_void_p]),
    "gpmdm_pf_read": (c_int, [c_void_p, _dp, _dp, _dp, c_void_p]),
    "gpmdm_pf_export": (c_int, [c_void_p, _dp, _i64p, _dp, _dp, _dp, _i64p, c_void_p]),
    "gpmdm_pf_enable_timing": (c_int, [c_void_p, c_int]),
    "gpmdm_pf_stage_times": (c_int, [c_void_p, _dp, _i64p]),
    "gpmdm_pf_set_dedup": (c_int, [c_void_p, c_int]),
    "gpmdm_pf_set_shard_order": (c_int, [c_void_p, c_int]),
    "gpmdm_pf_set_dyn_tiles": (c_int, [c_void_p, c_int]),
    "gpmdm_pf_timing_stages": (c_int, [c_void_p, ctypes.c_uint]),
    "gpmdm_pf_dyn_rows": (c_int, [c_void_p, _i64p, c_void_p]),
    "gpmdm_pf_frame": (c_int, [c_void_p, _i64p]),
    "gpmdm_pf_set_model": (c_int, [c_void_p, c_void_p]),
    "gpmdm_pf_health": (c_int, [c_void_p, _i64p, c_int, c_void_p]),
    "gpmdm_model_set_obs_cutoff": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_double, c_void_p]),
    "gpmdm_model_obs_cutoff": (c_int, [c_void_p, POINTER(ctypes.c_double)]),
    "gpmdm_model_build_obs_cutoff": (c_int, [c_void_p, ctypes.c_double, c_void_p, c_void_p, c_void_p]),
    "gpmdm_model_obs_cutoff_image": (c_int, [c_void_p, _i64p, c_void_p]),
    "gpmdm_pf_set_obs_cutoff": (c_int, [c_void_p, c_int]),
    "gpmdm_pf_set_obs_cutoff_split": (c_int, [c_void_p, c_int]),
    "gpmdm_pf_obs_cutoff_auto": (c_int, [c_void_p, POINTER(c_int), POINTER(ctypes.c_double)]),
    "gpmdm_pf_obs_cutoff_stats": (c_int, [c_void_p, _i64p, _i64p, c_int, c_void_p]),
    "gpmdm_pf_predict": (c_int, [c_void_p, _dp, c_void_p]),
    "gpmdm_pf_set_comm": (c_int, [c_void_p, c_void_p, c_int]),
    "gpmdm_comm_unique_id": (c_int, [c_void_p]),
    "gpmdm_comm_init": (c_int, [c_int, c_int, c_void_p, c_int, POINTER(c_void_p)]),
    "gpmdm_comm_destroy": (c_int, [c_void_p]),
    "gpmdm_comm_init_all": (c_int, [c_int, POINTER(c_int), POINTER(c_void_p)]),
    "gpmdm_comm_init_loopback": (c_int, [c_int, POINTER(c_int), POINTER(c_void_p)]),
    "gpmdm_pf_propagate_multi": (c_int, [POINTER(c_void_p), c_int, _dp, _dp, POINTER(c_void_p)]),
    "gpmdm_gp_factor": (c_int, [c_int, _dp, c_int64, c_int32, _dp, _dp, c_double, c_double, c_double,
                                _dp, c_int64, _dp, _dp]),
    "gpmdm_spd_inverse": (c_int, [c_int, c_void_p, c_int64, _dp, c_void_p]),
    "gpmdm_rng_walk_create": (c_int, [c_void_p, c_int64, POINTER(c_void_p)]),
    "gpmdm_rng_walk_reset": (c_int, [c_void_p, c_void_p, c_int64]),
    "gpmdm_rng_walk_state": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "gpmdm_rng_walk_states": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "gpmdm_rng_walk_destroy": (c_int, [c_void_p]),
    "gpmdm_last_error": (c_char_p, []),
    "gpmdm_version": (c_char_p, []),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def load():
    """Load libgpmdm_hip.so (once).  Raises RuntimeError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m gpmdm_amd.build` "
                           "(hipcc, gfx950).  There is no CPU fallback.")
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc == 0:
        return
    msg = load().gpmdm_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == -1:
        raise ValueError(text)
    raise RuntimeError(f"{text} (status {rc})")


def dptr(a):
    """double* of a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(_dp)


def i64ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(_i64p)
