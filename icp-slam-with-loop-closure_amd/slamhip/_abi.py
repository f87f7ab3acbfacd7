"""ctypes binding of libslamhip.so (the C-ABI declared in include/slamhip.h).

The library is built in-tree (``make -C icp-slam-with-loop-closure_amd/csrc``
or ``__graft_entry__.build()``) and loaded from this directory.  There is no
fallback: if the shared object is missing, or no ROCm GPU is visible when a
kernel is launched, the call raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SLAMHIP_LIB overrides the library path (A/B builds in diagnostics only)
LIB_PATH = os.environ.get("SLAMHIP_LIB") or os.path.join(_HERE, "libslamhip.so")

c_int = ctypes.c_int32
c_i64 = ctypes.c_int64
c_dbl = ctypes.c_double
c_ptr = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/slamhip.h one to one.
SIGNATURES = {
    "slam_abi_version": (c_int, []),
    "slam_last_error": (ctypes.c_char_p, []),
    "slam_icp_max_query_points": (c_int, []),
    "slam_icp_num_instances": (c_int, []),
    "slam_icp_instance_shape": (c_int, [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "slam_icp_force_instance": (c_int, [c_int]),
    "slam_icp_selected_instance": (c_int, [c_int]),
    "slam_icp_set_screen": (c_int, [c_int]),
    "slam_icp_set_schedule": (c_int, [c_int, c_int]),
    "slam_icp_set_stamps": (c_int, [c_ptr]),
    "slam_icp_set_schedule_heads": (c_int, [c_int]),
    "slam_icp_set_schedule_gangs": (c_int, [c_int, c_int]),
    "slam_icp_gang_timeouts": (c_int, []),
    "slam_icp_set_gang_wait": (c_int, [ctypes.c_uint32]),
    "slam_icp_set_gang_first_wait": (c_int, [ctypes.c_uint32]),
    "slam_icp_diag_occupy": (c_int, [c_int, ctypes.c_uint32, c_ptr]),
    "slam_icp_set_schedule_wide": (c_int, [c_int, c_int]),
    "slam_icp_set_bulk_gangs": (c_int, [c_int, c_int]),
    "slam_icp_set_schedule_warm": (c_int, [c_int]),
    "slam_icp_sched_sort": (c_int, [c_ptr, c_ptr, c_int, ctypes.c_float, c_ptr, c_ptr]),
    "slam_icp_set_sched_sort_one": (c_int, [c_int]),
    "slam_icp_set_tier_limit": (c_int, [c_int]),
    "slam_icp_set_xcd_map": (c_int, [c_int]),
    "slam_icp_set_angle_tier": (c_int, [c_int, ctypes.c_float]),
    "slam_icp_set_schedule_auto": (c_int, [c_int]),
    "slam_icp_set_drain": (c_int, [c_int]),
    "slam_icp_set_angle_tier_kind": (c_int, [c_int]),
    "slam_icp_set_angle_tier_mix": (c_int, [c_int, c_int]),
    "slam_icp_set_wide_groups": (c_int, [c_int]),
    "slam_icp_set_eval_counter": (c_int, [c_ptr]),
    "slam_icp_set_trace": (c_int, [c_ptr]),
    "slam_icp_status": (c_int, [c_ptr]),
    "slam_icp_batch_f64": (c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_dbl, c_int, c_dbl, c_int,
                                   c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr]),
    "slam_icp_step_f64": (c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_int, c_int, c_int,
                                  c_ptr, c_ptr, c_ptr, c_ptr, c_ptr]),
    "slam_kabsch2d_f64": (c_int, [c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr]),
    "slam_pgo_sgd_work_size": (c_i64, [c_int, c_int]),
    "slam_pgo_sgd_step_f64": (c_int, [c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_int, c_dbl, c_dbl, c_ptr, c_ptr]),
    "slam_pgo_orient_f64": (c_int, [c_ptr, c_int, c_ptr]),
    "slam_pgo_orient_from_tf_f64": (c_int, [c_ptr, c_int, c_ptr, c_ptr, c_ptr]),
    "slam_gn_work_size": (c_i64, [c_int, c_int, c_int]),
    "slam_gn_max_lds_band": (c_int, []),
    "slam_gn_set_stamps": (c_int, [c_ptr]),
    "slam_gn_set_solver": (c_int, [c_int]),
    "slam_gn_get_solver": (c_int, []),
    "slam_grid_work_size": (c_i64, [c_int, c_int, c_int]),
    "slam_grid_global_points_f64": (c_int, [c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr]),
    "slam_grid_update_i8": (c_int, [c_ptr, c_ptr, c_int, c_ptr, c_i64, c_dbl, c_dbl, c_dbl, c_int, c_int, c_int,
                                    c_int, c_ptr, c_ptr, c_ptr]),
    "slam_gn_bcr_block_rows": (c_int, [c_int, c_int]),
    "slam_gn_iteration_f64": (c_int, [c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
                                      c_ptr, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr]),
    "slam_gn_work_size_bordered": (c_i64, [c_int, c_int, c_int, c_int]),
    "slam_gn_iteration_bordered_f64": (c_int, [c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
                                               c_ptr, c_int, c_int, c_int, c_int, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
                                               c_ptr]),
    "slam_gn_iteration_schur_f64": (c_int, [c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
                                            c_ptr, c_int, c_int, c_int, c_int, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
                                            c_ptr, c_ptr]),
    "slam_gn_set_fused_back": (c_int, [c_int]),
    "slam_gn_get_fused_back": (c_int, []),
    "slam_gn_schur_supported": (c_int, []),
    "slam_gn_set_fused_wait": (c_int, [ctypes.c_uint32]),
}


class SlamHipError(RuntimeError):
    """A libslamhip entry point returned a negative status."""


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built: run `make -C {os.path.dirname(_HERE)}/csrc` "
                              "or __graft_entry__.build()")
        # Device pointers and streams come from PyTorch's HIP runtime: load it
        # first, so the library binds to that libamdhip64 instead of pulling in
        # a second copy (two runtimes in one process -> invalid pointers).
        import torch  # noqa: F401
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(handle, name):
                continue
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().slam_last_error().decode(errors="replace")
        raise SlamHipError(f"{what}: status {rc}: {msg}")
    return rc


def exported_symbols():
    """Names from SIGNATURES that the loaded library actually exports."""
    h = lib()
    return [n for n in SIGNATURES if hasattr(h, n)]
