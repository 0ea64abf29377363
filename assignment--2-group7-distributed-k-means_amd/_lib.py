"""ctypes binding of ``libkmeans_amd.so`` (C-ABI: ``include/kmeans_amd.h``).

Load order is pinned: ``torch`` (when importable) is imported first so the
dynamic linker binds the shim's ``libamdhip64.so.7`` / ``librccl.so.1`` to the
copies torch already mapped (same SONAMEs) and the process runs one HIP
runtime.  There is no CPU fallback: if the library or a gfx950 device is
missing, every entry point raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# KM_LIB: another build of the same sources (the diagnostic library, or an A/B
# variant from `make alt`), selected per process instead of copied over the
# product file (scripts/gpu_ab.sh)
LIB_PATH = os.environ.get("KM_LIB") or os.path.join(HERE, "libkmeans_amd.so")
ROOT = os.path.dirname(HERE)
HEADER = os.path.join(ROOT, "include", "kmeans_amd.h")

KM_ABI_VERSION = 6
KM_OK = 0
KM_EMPTY = 1

KM_K_ASSIGN, KM_K_RESOLVE, KM_K_STATS, KM_K_UPDATE, KM_K_PREP = range(5)
KERNEL_KINDS = {"assign": KM_K_ASSIGN, "resolve": KM_K_RESOLVE, "stats": KM_K_STATS, "update": KM_K_UPDATE,
                "prep": KM_K_PREP}


KM_STOP_CONVERGED, KM_STOP_EMPTY, KM_STOP_NONFINITE = 1, 2, 3
KM_MAX_BATCH = 32


class KmStatus(ctypes.Structure):
    _fields_ = [("sse", ctypes.c_double), ("max_shift", ctypes.c_double), ("n_empty", ctypes.c_int32),
                ("nonfinite", ctypes.c_int32), ("q_rerank", ctypes.c_int32), ("q_full", ctypes.c_int32),
                ("ran", ctypes.c_int32), ("stop_reason", ctypes.c_int32), ("repaired", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class KmInfo(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("d", ctypes.c_int32), ("dp", ctypes.c_int32), ("k", ctypes.c_int32),
                ("kp", ctypes.c_int32), ("path", ctypes.c_int32), ("n_cu", ctypes.c_int32),
                ("device", ctypes.c_int32), ("fused_stats", ctypes.c_int32),
                ("delta_stats", ctypes.c_int32)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_D = ctypes.c_double
_PD = ctypes.POINTER(ctypes.c_double)
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PF = ctypes.POINTER(ctypes.c_float)

# name -> argtypes (restype is always c_int except km_last_error)
SIGNATURES = {
    "km_abi_version": [],
    "km_device_count": [ctypes.POINTER(ctypes.c_int)],
    "km_create": [ctypes.c_int, ctypes.POINTER(_P)],
    "km_destroy": [_P],
    "km_set_stream": [_P, _P],
    "km_sync": [_P],
    "km_info_get": [_P, ctypes.POINTER(KmInfo)],
    "km_load_begin": [_P, _I64, _I32],
    "km_load_rows": [_P, _I64, _PF, _I64],
    "km_generate_blobs": [_P, _I64, _I32, _I64, _I32, ctypes.c_float, ctypes.c_float, ctypes.c_uint64],
    "km_sum_x": [_P, _PD],
    "km_set_sse": [_P, _I32],
    "km_set_screen": [_P, _I32],
    "km_get_screen": [_P, ctypes.POINTER(ctypes.c_int32)],
    "km_set_centroids": [_P, _PD, _I32, _I32],
    "km_get_centroids": [_P, _I32, _PD],
    "km_assign_stats": [_P],
    "km_stats_buffer": [_P, ctypes.POINTER(_P), _PI64],
    "km_bind_stats_buffer": [_P, _P],
    "km_update": [_P, ctypes.POINTER(KmStatus), _PI64],
    "km_batch_begin": [_P],
    "km_update_async": [_P, _D, _I64],
    "km_set_layout": [_P, _PI64, _I32, _I64, _I32],
    "km_repair_state": [_P, _PI32, _PI32],
    "km_repair_buffer": [_P, ctypes.POINTER(_P), _PI64],
    "km_bind_repair_buffer": [_P, _P],
    "km_repair_apply_async": [_P],
    "km_batch_end": [_P, ctypes.POINTER(KmStatus), _PI64, _PI32],
    "km_replace_rows": [_P, _PI32, _PD, _I32],
    "km_commit": [_P],
    "km_gather_rows": [_P, _PI64, _I32, _PD],
    "km_bernoulli_sample": [_P, ctypes.POINTER(ctypes.c_uint64), _PI64, _PI64, _I32, ctypes.c_double, _PI64,
                            ctypes.c_int64, _PI64],
    "km_predict": [_P, _PI32],
    "km_labels": [_P, _PI32],
    "km_profile": [_P, _I32],
    "km_profile_every": [_P, _I32],
    "km_prof_read": [_P, _I32, _PD, _PI64],
}

_lock = threading.Lock()
_lib = None


class KmError(RuntimeError):
    pass


def _pin_runtime():
    try:
        import torch  # noqa: F401  (binds libamdhip64.so.7 / librccl.so.1 first)
    except Exception:
        pass


def load(path: str = None):
    """Load (once) and return the ctypes library; raises RuntimeError if absent.
    ``path`` defaults to ``LIB_PATH`` as it is at the first call (diagnostic
    scripts point it at libkmeans_amd_diag.so before anything loads)."""
    global _lib
    path = path or LIB_PATH
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise KmError(f"HIP extension not built: {path} is missing "
                          f"(run `python -c 'import __graft_entry__ as g; g.build()'` or "
                          f"`make -C {os.path.join(HERE, 'csrc')}`)")
        _pin_runtime()
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        lib.km_last_error.argtypes = []
        lib.km_last_error.restype = ctypes.c_char_p
        _lib = lib
        return lib


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = load().km_last_error().decode(errors="replace")
        raise KmError(f"{what or 'kmeans_amd'} failed ({rc}): {msg}")
    return rc


def device_count() -> int:
    lib = load()
    n = ctypes.c_int(0)
    check(lib.km_device_count(ctypes.byref(n)), "km_device_count")
    return n.value


def exported_symbols():
    return list(SIGNATURES) + ["km_last_error"]
