"""ctypes binding of libspeedyml.so (include/speedy_ml.h).

The product path: every compute call goes to the hand-written gfx950 kernels in
this library.  There is no CPU fallback -- if the library is missing or no GPU is
visible, the compute entry points raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # speedy-ml-1_amd/
# SML_LIB: an alternative build of the same library (A/B measurements only)
LIB_PATH = os.environ.get("SML_LIB") or os.path.join(PKG_ROOT, "lib", "libspeedyml.so")
CSRC = os.path.join(PKG_ROOT, "csrc")

SML_OK = 0
SML_F32 = 1
SML_F64 = 2

# every symbol include/speedy_ml.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "sml_last_error", "sml_abi_version",
    "sml_spectral_create", "sml_spectral_destroy", "sml_spectral_tables",
    "sml_grid_batched", "sml_spec_batched", "sml_gridy_batched", "sml_gridx_batched",
    "sml_specx_batched", "sml_specy_batched", "sml_vdspec_batched", "sml_uvspec_batched",
    "sml_grid_host", "sml_spec_host",
    "sml_res_create", "sml_res_destroy", "sml_res_ninp", "sml_res_feedback_offsets",
    "sml_res_load_region_f32", "sml_res_load_region_f64", "sml_res_set_state", "sml_res_get_state",
    "sml_res_step", "sml_res_step_begin", "sml_res_step_finish", "sml_res_step_finish_grid", "sml_res_step_finish_assemble", "sml_res_step_host", "sml_res_synchronize",
    "sml_res_footprint", "sml_res_enable_timing", "sml_res_kernel_times", "sml_res_set_read_waves",
    "sml_res_set_begin_mode", "sml_res_begin_fused",
    "sml_exchange_assemble",
    "sml_res_tile_inputs", "sml_res_tile_feedback", "sml_res_tile_local_model",
    "sml_nc_read_region", "sml_nc_write_region",
    "sml_dyn_create", "sml_dyn_destroy", "sml_dyn_impint", "sml_dyn_set_forcing", "sml_dyn_set_state",
    "sml_dyn_get_state", "sml_dyn_get_phi", "sml_dyn_get_tendencies", "sml_dyn_state_device",
    "sml_dyn_step", "sml_dyn_step_host", "sml_dyn_leapfrog", "sml_dyn_window", "sml_dyn_from_grid", "sml_dyn_to_grid",
    "sml_dyn_is_safe", "sml_dyn_from_grid_host", "sml_dyn_to_grid_host",
    "sml_dyn_set_physics", "sml_dyn_set_clock", "sml_dyn_get_clock", "sml_dyn_set_rad_state",
    "sml_dyn_get_rad_state", "sml_dyn_phypar", "sml_dyn_phypar_host", "sml_dyn_sol_oz", "sml_phys_sflset",
    "sml_train_create", "sml_train_destroy", "sml_train_reset", "sml_train_accumulate", "sml_train_solve",
    "sml_train_npad", "sml_train_get_gram", "sml_probe_mfma_f64",
    "sml_stream_create_cu_range", "sml_stream_destroy",
    "sml_dyn_run_model", "sml_dyn_last_safe", "sml_dyn_set_check_cus", "sml_res_info",
    "sml_comm_unique_id", "sml_comm_create", "sml_comm_create_file", "sml_comm_destroy", "sml_comm_rank",
    "sml_comm_allgather",
    "sml_hybrid_create", "sml_hybrid_destroy", "sml_hybrid_set_buffers", "sml_hybrid_set_tisr",
    "sml_hybrid_streams", "sml_hybrid_cus", "sml_hybrid_start", "sml_hybrid_predict", "sml_hybrid_advance", "sml_hybrid_step",
    "sml_hybrid_run_speedy", "sml_hybrid_sync",
    "sml_device_alloc", "sml_device_free", "sml_copy_to_device", "sml_copy_to_host", "sml_region_geometry",
    "sml_processor_decomposition", "sml_hybrid_set_tisr_table", "sml_tisr_date_index", "sml_res_tile_tisr_field",
    "sml_res_create_generic", "sml_res_step_slab", "sml_res_start_prediction",
    "sml_comm_create_local", "sml_exchange_plan", "sml_hybrid_advance_slabs", "sml_hybrid_set_hop_mode",
    "sml_hybrid_hop_mode", "sml_calendar_delta_hour", "sml_hybrid_set_feb29", "sml_hybrid_get_feb29",
    "sml_res_mean_std", "sml_res_set_outvec_ld", "sml_hybrid_set_slab", "sml_hybrid_start_slab",
    "sml_hybrid_exchange_width", "sml_hybrid_slab_buffers", "sml_dyn_set_hybrid_sst", "sml_dyn_set_sea_ice",
    "sml_hybrid_set_pipelined", "sml_res_step_cancel", "sml_res_step_begun", "sml_hybrid_set_force_exchange",
    "sml_hybrid_exchanges", "sml_hybrid_set_chain", "sml_hybrid_chain", "sml_hybrid_exchange_stream",
    "sml_res_set_update_cus", "sml_res_update_balanced", "sml_probe_mfma_f64_clock", "sml_res_ell_layout",
    "sml_dyn_get_sea_ice", "sml_dyn_get_physics", "sml_dyn_get_forcing", "sml_dyn_set_surface",
    "sml_dyn_set_climatology", "sml_dyn_fordate", "sml_dyn_fordate_ex", "sml_dyn_fordate_count",
    "sml_hybrid_set_calendar", "sml_hybrid_window_date", "sml_hybrid_set_hop_timeout",
    "sml_dyn_set_check_timeout", "sml_dyn_check_stream", "sml_dyn_set_fused", "sml_res_set_reference_paths",
    "sml_train_set_panel",
)

SML_HOP_AUTO, SML_HOP_WAIT_VALUE, SML_HOP_EVENTS, SML_HOP_KERNEL = 0, 1, 2, 3
SML_CHAIN_AUTO, SML_CHAIN_TWO_STREAMS, SML_CHAIN_SPEEDY = 0, 1, 2
SML_RES_PATH_CSR, SML_RES_PATH_PER_REGION, SML_RES_PATH_UNGROUPED_FINISH = 1, 2, 4


class SmlError(RuntimeError):
    pass


_lib = None


def build(jobs: int = 8) -> str:
    """Compile libspeedyml.so for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", CSRC, f"-j{jobs}"], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SmlError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != SML_OK:
        msg = lib().sml_last_error().decode(errors="replace")
        raise SmlError(f"libspeedyml error {rc}: {msg}")


def _declare(L: ctypes.CDLL) -> None:
    vp, i, d, i64p = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_int64)
    pp = ctypes.POINTER(ctypes.c_void_p)
    ip = ctypes.POINTER(ctypes.c_int)
    L.sml_last_error.restype = ctypes.c_char_p
    L.sml_last_error.argtypes = []
    L.sml_abi_version.restype = i
    sig = {
        "sml_spectral_create": [d, pp],
        "sml_spectral_destroy": [vp],
        "sml_spectral_tables": [vp, vp, vp, vp, vp],
        "sml_grid_batched": [vp, vp, vp, i, i, vp],
        "sml_spec_batched": [vp, vp, vp, i, vp],
        "sml_gridy_batched": [vp, vp, vp, i, vp],
        "sml_gridx_batched": [vp, vp, vp, i, i, vp],
        "sml_specx_batched": [vp, vp, vp, i, vp],
        "sml_specy_batched": [vp, vp, vp, i, vp],
        "sml_vdspec_batched": [vp, vp, vp, vp, vp, i, i, vp],
        "sml_uvspec_batched": [vp, vp, vp, vp, vp, i, vp],
        "sml_grid_host": [vp, vp, vp, i, i],
        "sml_spec_host": [vp, vp, vp, i],
        "sml_res_create": [i, i, vp, vp, vp, vp, i, i, i, d, pp],
        "sml_res_destroy": [vp],
        "sml_res_ninp": [vp, i, ctypes.POINTER(ctypes.c_int)],
        "sml_res_feedback_offsets": [vp, vp],
        "sml_res_load_region_f32": [vp, i, vp, vp, vp, vp, vp, vp, vp],
        "sml_res_load_region_f64": [vp, i, vp, vp, vp, vp, vp, vp, vp],
        "sml_res_set_state": [vp, i, vp],
        "sml_res_get_state": [vp, i, vp],
        "sml_res_step": [vp, vp, vp, vp, vp],
        "sml_res_step_begin": [vp, vp, vp],
        "sml_res_step_finish": [vp, vp, vp, vp],
        "sml_res_step_finish_grid": [vp, vp, vp, vp, vp, vp],
        "sml_res_step_finish_assemble": [vp, vp, vp, vp, vp, vp, vp, vp, vp],
        "sml_res_step_host": [vp, vp, vp, vp],
        "sml_res_synchronize": [vp, vp, i, ctypes.c_int64, vp],
        "sml_res_footprint": [vp, i64p, i64p],
        "sml_res_enable_timing": [vp, i],
        "sml_res_set_read_waves": [vp, i],
        "sml_res_set_begin_mode": [vp, i],
        "sml_hybrid_set_pipelined": [vp, i],
        "sml_res_begin_fused": [vp, vp],
        "sml_res_kernel_times": [vp, vp, vp, i, ctypes.POINTER(ctypes.c_int)],
        "sml_exchange_assemble": [vp, vp, vp, vp, vp, vp],
        "sml_res_tile_inputs": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
        "sml_res_tile_feedback": [vp, vp, vp, vp, vp, vp, vp],
        "sml_res_tile_local_model": [vp, vp, vp, vp, vp],
        "sml_nc_read_region": [ctypes.c_char_p, vp, vp, vp, vp, vp, vp, vp, vp],
        "sml_nc_write_region": [ctypes.c_char_p, i, i, i, i, i, vp, vp, vp, vp, vp, vp, vp],
        "sml_dyn_create": [d, pp],
        "sml_dyn_destroy": [vp],
        "sml_dyn_impint": [vp, d, d],
        "sml_dyn_set_forcing": [vp, vp, vp, vp],
        "sml_dyn_set_state": [vp, vp, vp, vp, vp, vp],
        "sml_dyn_get_state": [vp, vp, vp, vp, vp, vp],
        "sml_dyn_get_phi": [vp, vp],
        "sml_dyn_get_tendencies": [vp, vp],
        "sml_dyn_state_device": [vp, pp, pp],
        "sml_dyn_step": [vp, i, i, d, d, d, d, vp, vp],
        "sml_dyn_step_host": [vp, i, i, d, d, d, d, vp],
        "sml_dyn_leapfrog": [vp, i, d, d, d, d, vp, vp],
        "sml_dyn_window": [vp, i, d, d, d, d, vp],
        "sml_dyn_from_grid": [vp, vp, vp, vp, vp],
        "sml_dyn_to_grid": [vp, vp, vp, vp],
        "sml_dyn_is_safe": [vp],
        "sml_dyn_from_grid_host": [vp, vp, vp, vp, ctypes.POINTER(ctypes.c_int)],
        "sml_dyn_to_grid_host": [vp, vp, vp],
        "sml_dyn_set_physics": [vp, vp],
        "sml_dyn_set_clock": [vp, i, i],
        "sml_dyn_get_clock": [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
        "sml_dyn_set_rad_state": [vp, vp],
        "sml_dyn_get_rad_state": [vp, vp],
        "sml_dyn_phypar": [vp, vp, vp, vp, vp, vp, vp, i, vp, vp],
        "sml_dyn_phypar_host": [vp, vp, vp, vp, vp, vp, vp, i, vp],
        "sml_dyn_sol_oz": [vp, d, vp],
        "sml_phys_sflset": [vp, vp],
        "sml_train_create": [i, vp, i, pp],
        "sml_train_destroy": [vp],
        "sml_train_reset": [vp, vp],
        "sml_train_accumulate": [vp, vp, vp, i, vp],
        "sml_train_solve": [vp, i, d, d, i, d, vp, vp, vp],
        "sml_train_npad": [vp, ctypes.POINTER(ctypes.c_int)],
        "sml_train_get_gram": [vp, i, vp, vp],
        "sml_probe_mfma_f64": [i, ctypes.POINTER(ctypes.c_double)],
        "sml_stream_create_cu_range": [i, i, pp],
        "sml_stream_destroy": [vp],
        "sml_dyn_run_model": [vp, vp, vp, i, d, d, d, d, vp, vp, vp],
        "sml_dyn_last_safe": [vp, ip, vp],
        "sml_dyn_set_check_cus": [vp, i, i],
        "sml_dyn_set_check_timeout": [vp, ctypes.c_int64],
        "sml_dyn_check_stream": [vp, pp],
        "sml_dyn_set_fused": [vp, i],
        "sml_res_set_reference_paths": [vp, i],
        "sml_train_set_panel": [vp, i],
        "sml_res_info": [vp, ip, ip, ip, ip, vp],
        "sml_comm_unique_id": [vp],
        "sml_comm_create": [i, i, vp, pp],
        "sml_comm_create_file": [i, i, ctypes.c_char_p, i, pp],
        "sml_comm_destroy": [vp],
        "sml_comm_rank": [vp, ip, ip],
        "sml_comm_allgather": [vp, vp, vp, ctypes.c_int64, vp],
        "sml_hybrid_create": [vp, vp, vp, i, d, d, d, d, i, i, pp],
        "sml_hybrid_destroy": [vp],
        "sml_hybrid_set_buffers": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
        "sml_hybrid_set_tisr": [vp, vp],
        "sml_hybrid_streams": [vp, pp, pp],
        "sml_hybrid_cus": [vp, ip, ip],
        "sml_hybrid_start": [vp, vp, vp, vp, vp, vp],
        "sml_hybrid_predict": [vp],
        "sml_hybrid_advance": [vp, vp],
        "sml_hybrid_step": [vp],
        "sml_hybrid_run_speedy": [vp, ip],
        "sml_hybrid_sync": [vp],
        "sml_device_alloc": [ctypes.c_int64, pp],
        "sml_device_free": [vp],
        "sml_copy_to_device": [vp, vp, ctypes.c_int64],
        "sml_copy_to_host": [vp, vp, ctypes.c_int64],
        "sml_region_geometry": [i, i, ip],
        "sml_processor_decomposition": [i, i, i, ip, ip],
        "sml_hybrid_set_tisr_table": [vp, vp, i, i, ctypes.c_int64, i],
        "sml_tisr_date_index": [i, ctypes.c_int64, ip, ip],
        "sml_res_tile_tisr_field": [vp, vp, vp, vp],
        "sml_res_create_generic": [i, i, vp, vp, vp, vp, i, i, vp, i, d, pp],
        "sml_res_step_slab": [vp, vp, vp, vp, vp, vp],
        "sml_res_start_prediction": [vp, vp, i, ctypes.c_int64, vp, vp],
        "sml_comm_create_local": [i, i, pp],
        "sml_exchange_plan": [i, i, ip, ip, vp],
        "sml_hybrid_advance_slabs": [vp, vp],
        "sml_hybrid_set_hop_mode": [vp, i],
        "sml_hybrid_hop_mode": [vp, ip, ip],
        "sml_calendar_delta_hour": [i, ctypes.c_int64, ip, ip],
        "sml_hybrid_set_feb29": [vp, i],
        "sml_hybrid_get_feb29": [vp, ip],
        "sml_res_mean_std": [vp, i, vp, vp],
        "sml_res_set_outvec_ld": [vp, i],
        "sml_hybrid_set_slab": [vp, vp, vp, vp, i, i, d],
        "sml_hybrid_start_slab": [vp, vp],
        "sml_hybrid_exchange_width": [vp, ip],
        "sml_hybrid_slab_buffers": [vp, pp, pp, ip, pp, pp],
        "sml_dyn_set_hybrid_sst": [vp, vp, d, vp],
        "sml_dyn_set_sea_ice": [vp, vp, vp],
        "sml_res_step_cancel": [vp],
        "sml_res_step_begun": [vp, ip],
        "sml_hybrid_set_force_exchange": [vp, i],
        "sml_hybrid_exchanges": [vp, i64p],
        "sml_hybrid_set_chain": [vp, i],
        "sml_hybrid_chain": [vp, ip, ip],
        "sml_hybrid_exchange_stream": [vp, pp],
        "sml_res_set_update_cus": [vp, i],
        "sml_res_update_balanced": [vp, ip],
        "sml_res_ell_layout": [vp, i, ip, ip, ip, ip],
        "sml_probe_mfma_f64_clock": [i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)],
        "sml_dyn_get_sea_ice": [vp, vp, vp],
        "sml_dyn_get_physics": [vp, vp],
        "sml_dyn_get_forcing": [vp, vp, vp, vp],
        "sml_dyn_set_surface": [vp, vp],
        "sml_dyn_set_climatology": [vp, vp],
        "sml_dyn_fordate": [vp, i, i, i, vp],
        "sml_dyn_fordate_ex": [vp, i, i, i, i, vp],
        "sml_dyn_fordate_count": [vp, ip],
        "sml_hybrid_set_calendar": [vp, i, ctypes.c_int64, i],
        "sml_hybrid_window_date": [vp, ip],
        "sml_hybrid_set_hop_timeout": [vp, ctypes.c_int64],
    }
    for name, args in sig.items():
        if os.environ.get("SML_LIB") and not hasattr(L, name):
            continue  # an older build for an A/B: entry points added since are absent
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = i


def ptr(x) -> ctypes.c_void_p:
    """Address of a numpy array or a torch tensor (device or host); None -> NULL."""
    if x is None:
        return ctypes.c_void_p(0)
    if hasattr(x, "data_ptr"):
        return ctypes.c_void_p(x.data_ptr())
    if hasattr(x, "ctypes"):
        return x.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(int(x))


def stream_ptr(stream) -> ctypes.c_void_p:
    """hipStream_t of a torch stream (None -> torch's current stream)."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
