"""ctypes binding of libdmlp.so (the in-tree native core).

The library is loaded from the package directory only; if it is missing we raise instead of
silently falling back to a Python path (GPU code must be the native HIP code).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "libdmlp.so"

_lib = None

vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_int64, C.c_float
i64p = C.POINTER(C.c_int64)
i32p = C.POINTER(C.c_int)

_SIGS = {
    "dmlp_center": (i32, [vp, i64, i32, vp, vp]),
    "dmlp_prep_data": (i32, [vp, i64, i32, vp, i32, vp, vp, vp, vp, vp]),
    "dmlp_prep_queries": (i32, [vp, i64, i32, vp, i32, vp, vp, vp, vp, vp]),
    "dmlp_host_threads": (i32, []),
    "dmlp_cpu_center": (None, [vp, i64, i32, vp]),
    "dmlp_cpu_prep_queries": (i32, [vp, i64, i32, vp, i32, vp, vp]),
    "dmlp_cpu_prep_data": (i32, [vp, i64, i32, vp, i32, vp, vp, vp]),
    "dmlp_d2h_async": (i32, [vp, vp, i64, vp]),
    "dmlp_cpu_prep_data_tiles": (i32, [vp, i64, i32, vp, i32, i64, i64, vp, vp, vp]),
    "dmlp_host_ops_h2d": (i32, [vp, i64, vp, i64, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                vp, i32, vp]),
    "dmlp_cpu_center_rows": (None, [vp, i64, i32, vp]),
    "dmlp_cpu_prep_queries_rows": (i32, [vp, i64, i32, vp, i32, vp, vp]),
    "dmlp_cpu_prep_data_tiles_rows": (i32, [vp, i64, i32, vp, i32, i64, i64, vp, vp, vp]),
    "dmlp_cpu_rows_i32_rows": (i32, [vp, i64, i32, vp]),
    "dmlp_cpu_gather_rows": (None, [vp, i64, i32, vp]),
    "dmlp_cpu_rows_i32": (i32, [vp, i64, vp]),
    "dmlp_rows_from_i32": (i32, [vp, i64, vp, vp]),
    "dmlp_render_rows": (i32, [i32, i32, vp, vp, i64, i64, i64, vp, vp, i32, vp, vp, vp, vp, vp, vp,
                               vp, vp]),
    "dmlp_host_ops_h2d_tiles": (i32, [vp, i64, i64, i64, vp, i64, i32, vp, i32, vp, vp, vp, vp, vp,
                                      vp, vp, vp, vp, vp, i32, vp]),
    "dmlp_screen_kmax": (i32, [i32]),
    "dmlp_screen_lds_bytes": (i32, [i32, i32]),
    "dmlp_screen_waves": (i32, [i32, i32]),
    "dmlp_set_screen_mode": (None, [i32]),
    "dmlp_set_stream_mode": (None, [i32]),
    "dmlp_set_stream_groups": (None, [i32]),
    "dmlp_screen_stream_cap": (i32, [i32]),
    "dmlp_set_stream_sub": (None, [i32]),
    "dmlp_screen_stream_kmax": (i32, []),
    "dmlp_screen_stream_waves_per_cu": (i32, [i32]),
    "dmlp_stream_debug_counters": (i32, [vp, i32]),
    "dmlp_screen_stream_qw": (i32, [i32]),
    "dmlp_screen_stream": (i32, [i32, vp, vp, i64, vp, vp, vp, vp, vp, i32, i32, vp, vp, f32, i32, vp,
                                 vp, vp]),
    "dmlp_screen_debug_counters": (i32, [vp, i32]),
    "dmlp_screen_x1_kmax": (i32, []),
    "dmlp_screen_x1_qw": (i32, [i32]),
    "dmlp_screen_x1_cols": (i32, [i32, i32]),
    "dmlp_screen_x1_cap": (i32, [i32]),
    "dmlp_screen_x1_cap_kt": (i32, [i32, i32]),
    "dmlp_screen_x1_waves_per_cu": (i32, [i32]),
    "dmlp_screen_x1_waves_per_cu_kt": (i32, [i32, i32]),
    "dmlp_screen_x1_min_slices": (i64, [i64]),
    "dmlp_screen_x1_bound": (None, [i32, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "dmlp_screen_x1_bound2": (None, [i32, i32, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                     C.POINTER(C.c_float)]),
    "dmlp_screen_x1": (i32, [i32, i32, i32, vp, vp, i64, i64, vp, vp, vp, vp, i32, i32, vp, vp, i32,
                             vp, vp, vp, vp]),
    "dmlp_screen_x1_early": (i32, [i32, i32, vp, vp, i64, i64, vp, vp, vp, vp, i32, i32, vp, vp,
                                   i32, i32, vp, vp, vp, vp, vp]),
    "dmlp_screen_x1_group_rows": (i32, [i32]),
    "dmlp_screen_x1_part": (i32, [i32, i32, i32, vp, vp, i64, i64, vp, vp, vp, vp, i32, i32, vp, vp,
                                  i32, i32, i32, vp, vp, vp, vp]),
    "dmlp_refine_groups": (i32, [i32, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, i32, i32, i64, vp, vp, i32, vp, vp, i32, vp, i32, i32, vp, vp, vp, vp, vp]),
    "dmlp_refine_groups2": (i32, [i32, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, i32, i32, i64, vp, vp, i32, vp, vp, i32, vp, i32, i32, vp, vp, vp, vp, i32, vp]),
    "dmlp_x1_seed": (i32, [vp, vp, i32, i32, vp, vp]),
    "dmlp_arena_reserve": (i32, [i64, i64]),
    "dmlp_knn_local": (i32, [vp, i64, i32, vp, i64, vp, i32, vp, vp, vp, i32, i32, vp, vp, i32, vp]),
    "dmlp_step": (i32, [vp]),
    "dmlp_step_emit": (i32, [vp, i64, vp]),
    "dmlp_step_early": (None, [i32]),
    "dmlp_step_early_delay": (None, [i32]),
    "dmlp_step_events": (i32, [i32]),
    "dmlp_step_timeline": (i32, [vp, vp, i32]),
    "dmlp_pipeline_set": (i32, [C.c_char_p, i32]),
    "dmlp_pipeline_stats": (None, [vp]),
    "dmlp_screen_x1_collect": (i32, [i32, i32, vp, vp, i64, i64, vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, vp, vp, vp, vp]),
    "dmlp_screen": (i32, [i32, i32, vp, vp, i64, vp, vp, vp, vp, vp, i32, vp, vp, f32, i32, vp,
                          vp, vp]),
    "dmlp_screen_hl": (i32, [i32, i32, i32, i32, vp, vp, i64, vp, vp, vp, vp, vp, i32, vp, vp,
                             f32, i32, vp, vp, vp]),
    "dmlp_screen_waves_hl": (i32, [i32, i32, i32]),
    "dmlp_screen_lds_bytes_hl": (i32, [i32, i32, i32]),
    "dmlp_refine": (i32, [i32, vp, vp, i32, vp, i32, vp, vp, vp, i32, vp, vp, i32, vp, i32, i32, vp, vp, vp, vp, vp]),
    "dmlp_exact_rows": (i32, [vp, i64, i32, vp, vp, i32, vp, i64, vp]),
    "dmlp_fallback_bytes": (i64, [i32, i64]),
    "dmlp_fallback_select_kmax": (i32, []),
    "dmlp_exact_topk_kmax": (i32, []),
    "dmlp_exact_topk_kmax_for": (i32, [i64]),
    "dmlp_exact_topk": (i32, [vp, i64, i32, vp, vp, vp, i32, i32, vp, vp, i32, vp]),
    "dmlp_exact_f64_amax": (i32, []),
    "dmlp_exact_f64_kmax": (i32, []),
    "dmlp_exact_f64_bytes": (i64, [i64, i32, i32, i32]),
    "dmlp_exact_f64": (i32, [vp, i64, i32, vp, vp, vp, i32, i32, vp, vp, i32, vp, vp, vp, i64, vp]),
    "dmlp_exact_f64_probe": (i32, [vp, i64, i32, vp, vp, vp, i64, vp]),
    "dmlp_exact_f64_layout": (None, [i64, i32, i32, i32, vp]),
    "dmlp_fallback_select_bytes": (i64, [i32, i64]),
    "dmlp_fallback_select": (i32, [vp, i64, i32, vp, vp, vp, i32, vp, i64, vp, vp, i32, vp]),
    "dmlp_fallback_topk": (i32, [vp, i64, i32, vp, vp, vp, i32, vp, i64, vp, vp, i32, vp]),
    "dmlp_merge": (i32, [vp, vp, i32, i64, i32, vp, i32, vp, vp, i32, vp]),
    "dmlp_finalize": (i32, [vp, vp, i32, vp, vp, i32, vp, i32, i32, vp, vp, vp]),
    "dmlp_format_bound": (i64, [i32]),
    "dmlp_format_scratch": (i64, [i32]),
    "dmlp_format_report": (i32, [vp, i32, i32, vp, vp, vp]),
    "dmlp_cpu_knn": (i32, [vp, i64, i32, vp, i64, vp, i32, vp, vp, i32]),
    "dmlp_cpu_finalize": (i32, [vp, vp, i32, vp, i64, vp, vp, vp]),
    "dmlp_cpu_merge": (i32, [vp, vp, i32, i64, i32, vp, i64, vp, vp, i32]),
    "dmlp_kdtree_knn": (i32, [vp, i64, i32, vp, i64, vp, i32, vp, vp]),
    "dmlp_cpu_format_report": (i64, [vp, i64, i64, vp]),
    "dmlp_cpu_write_input": (i32, [C.c_char_p, vp, vp, i64, vp, vp, i64, i32]),
    "dmlp_cpu_i32_range": (None, [vp, i64, i32p, i32p]),
    "dmlp_host_i32_range": (None, [vp, i64, i32p, i32p]),
    "dmlp_atomic_fetch_add_i64": (i64, [vp, i64]),
    "dmlp_atomic_store_i64": (None, [vp, i64]),
    "dmlp_cpu_format_debug": (i64, [vp, vp, i32, vp, vp, i64, vp, i64]),
    "dmlp_parse_header": (i32, [vp, i64, i64p, i64p, i32p, i64p]),
    "dmlp_parse_body": (i64, [vp, i64, i64, i64, i64, i32, vp, vp, vp, vp, i32]),
    "dmlp_version": (C.c_char_p, []),
    "dmlp_device_count": (i32, []),
    "dmlp_plane_slices": (i32, []),
    "dmlp_plane_bytes": (i64, [i64, i32, i32]),
    "dmlp_plane_init": (i32, [vp, i64, i64, i32, i32]),
    "dmlp_plane_slice": (i32, [i64, i32, i32, i64p, i64p]),
    "dmlp_plane_regions": (i32, [vp, i64, i32, vp, vp, vp, vp]),
    "dmlp_plane_put_mu": (i32, [vp, i32, vp]),
    "dmlp_plane_get_mu": (i32, [vp, i32, vp]),
    "dmlp_plane_render": (i32, [vp, vp, vp, i64, i32, vp, i32, i32]),
    "dmlp_plane_wait": (i32, [vp, i32, i32, i32p, C.POINTER(C.c_float)]),
    "dmlp_plane_ready": (i32, [vp, i32, i32]),
    "dmlp_host_register": (i32, [vp, i64]),
    "dmlp_host_device_view": (vp, [vp, i64, vp]),
    "dmlp_host_unregister": (i32, [vp]),
}


class NativeLibraryMissing(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes handle of libdmlp.so."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        if os.environ.get("DMLP_AUTOBUILD", "1") == "1":
            from . import build as _build
            _build.build(engine=False)
        if not LIB_PATH.exists():
            raise NativeLibraryMissing(
                f"{LIB_PATH} not built; run `python -m distributed_machine_learning_project_amd.build`")
    # DMLP_LIB: an alternative build of the same library (kernel A/B runs on one box)
    h = C.CDLL(os.environ.get("DMLP_LIB") or str(LIB_PATH), mode=C.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    _lib = h
    return h


def i32_range(a) -> tuple[int, int]:
    """(min, max) of an int32 numpy array (one native pass); (0, -1) when empty."""
    import numpy as np
    a = np.ascontiguousarray(a, np.int32)
    if a.size == 0:
        return 0, -1
    lo, hi = C.c_int(), C.c_int()
    lib().dmlp_cpu_i32_range(a.ctypes.data, a.size, C.byref(lo), C.byref(hi))
    return lo.value, hi.value


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")
    return rc
