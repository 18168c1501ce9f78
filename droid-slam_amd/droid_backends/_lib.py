"""ctypes binding of libdroid_hip.so (declarations mirror include/droid_backends.h)."""
import ctypes
import os

import torch  # noqa: F401  (loads torch's HIP runtime first; the library shares it)

_HERE = os.path.dirname(os.path.abspath(__file__))
# DROID_HIP_LIB points at an alternative build (kernel A/B experiments)
LIB_PATH = os.environ.get("DROID_HIP_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libdroid_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "droid_backends: HIP library %s is missing - run `python -c \"import __graft_entry__ as g; "
        "g.build()\"` (or `make -C droid-slam_amd/csrc`) first" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

_p = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t

_SIGS = {
    "droid_last_error": ([], ctypes.c_char_p),
    "droid_build_info": ([], ctypes.c_int),
    "droid_abi_version": ([], _i),
    "droid_device_count": ([], _i),
    "droid_corr_index_forward": ([_i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p], _i),
    "droid_corr_index_backward": ([_i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p], _i),
    "droid_corr_pyramid_lookup": ([_i, _p, _p, _p, _i, _p, _p, _i, _i, _i, _i, _p], _i),
    "droid_corr_pyramid_lookup_tiled": ([_p, _p, _p, _p, _i, _p, _p, _i, _i, _i, _p], _i),
    "droid_corr_pyramid_lookup_nhwc": ([_p, _p, _p, _i, _p, _p, _i, _i, _i, _i, _p], _i),
    "droid_corr_lookup_ce0": ([_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_corr_lookup_ce0_tiled": ([_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_corr_lookup_ce0_tiled_slots": ([_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_corr_volume_pyramid": ([_p, _p, _p, _i, _i, _i, _i, _p, _i, _p], _i),
    "droid_corr_alt_ce0": ([_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_corr_alt_ce0_ordered": ([_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_conv_nhwc_f16": ([_p, _p, _p, _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _i, _i,
                             _p, _i, _p, _i, _p, _p, _i, _p, _p], _i),
    "droid_conv_gru_pre_f16": ([_p, _p, _p, _i, _p, _p, _p, _i, _i, _i, _i, _i, _p, _i, _i, _p, _i, _p, _i,
                                _p, _p, _i, _p, _p, _i, _i, _p], _i),
    "droid_conv_wino_f16": ([_p, _p, _p, _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _i, _i, _p, _i, _p, _i,
                             _p, _p, _i, _p, _p, _i, _i, _p], _i),
    "droid_transpose_f16": ([_p, _p, _i, _i, _i, _i, _p], _i),
    "droid_conv1x1_nchw_f16": ([_p, _i, _p, _i, _p, _p, _i, _i, _i, _p], _i),
    "droid_conv_dw_head_f16": ([_p, _p, _p, _i, _p, _p, _i, _i, _i, _p, _p, _p], _i),
    "droid_flow_enc0_f16": ([_p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_gru_global_f16": ([_p, _p, _p, _p, _i, _i, _p], _i),
    "droid_gru_global_split_f16": ([_p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_glo_gates_f32": ([_p, _i, _p, _p, _p, _p, _i, _p], _i),
    "droid_head_finish_f32": ([_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p], _i),
    "droid_eta_damping_f32": ([_p, _p, _p, _p, _p, _i, _i, ctypes.c_float, _p], _i),
    "droid_segment_mean_f16": ([_p, _p, _p, _p, _i, ctypes.c_long, _p], _i),
    "droid_altcorr_forward": ([_i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p], _i),
    "droid_altcorr_backward": ([_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p], _i),
    "droid_projective_transform": ([_p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p], _i),
    "droid_frame_distance": ([_p, _p, _p, _p, _p, _i, _i, _i, _f, _p, _p], _i),
    "droid_instance_norm_workspace": ([_i, _i, _i], _sz),
    "droid_instance_norm_act_f16": ([_p, _p, _p, _i, _i, _i, _i, _f, _p, _sz, _p], _i),
    "droid_proximity_workspace": ([_i, _i, _i], _sz),
    "droid_proximity_select": ([_p, _i, _i, _i, _i, _i, _f, _p, _p, _i, _i, _i, _p, _p, _p, _p, _sz, _p], _i),
    "droid_projmap": ([_p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p], _i),
    "droid_iproj": ([_p, _p, _p, _i, _i, _i, _p, _p], _i),
    "droid_depth_filter": ([_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p], _i),
    "droid_ba_plan_create": ([_p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, ctypes.POINTER(_p)], _i),
    "droid_ba_plan_create_sharded": ([_p, _p, _i, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                                      ctypes.POINTER(_p)], _i),
    "droid_ba_plan_order": ([_p, ctypes.POINTER(_i), _p, ctypes.POINTER(_i), ctypes.POINTER(_i)], _i),
    "droid_ba_plan_flag_offset": ([_p, ctypes.POINTER(_sz)], _i),
    "droid_ba_plan_clear_status": ([_p, _p, _p], _i),
    "droid_ba_plan_destroy": ([_p], None),
    "droid_ba_plan_workspace_bytes": ([_p], _sz),
    "droid_ba_set_order": ([_i], _i),
    "droid_ba_plan_info": ([_p, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i),
                            ctypes.POINTER(_i)], _i),
    "droid_ba_plan_kx": ([_p, _p], _i),
    "droid_ba_plan_system_region": ([_p, ctypes.POINTER(_sz), ctypes.POINTER(_sz)], _i),
    "droid_ba_plan_ints_region": ([_p, ctypes.POINTER(_sz), ctypes.POINTER(_sz)], _i),
    "droid_ba_plan_upload": ([_p, _p, _p], _i),
    "droid_ba_build_system": ([_p, _p, _p, _p, _p, _p, _p, _p, _p, _p], _i),
    "droid_ba_solve_update": ([_p, _p, _p, _p, _p, _p, _p, _p, _p, _f, _f, _p, _p, _p], _i),
    "droid_ba_solve_system": ([_p, _p, _f, _f, _p, _p], _i),
    "droid_ba_apply_update": ([_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p], _i),
    "droid_chol_plan_create": ([_i, ctypes.POINTER(_p)], _i),
    "droid_chol_plan_info": ([_p, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i),
                              ctypes.POINTER(_i)], _i),
    "droid_chol_set_system": ([_p, _p, _p, _i, _p, _p], _i),
    "droid_chol_solve": ([_p, _p, _f, _f, _p, _p], _i),
    "droid_chol_plan_tasks": ([_p, _p], _i),
    "droid_chol_plan_structure": ([_p, _p, _p, _p, _p], _i),
    "droid_ba_run": ([_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _f, _f, _p, _p, _p], _i),
}

# the testing builds' hooks (include/droid_backends_testing.h): bound when the
# loaded library exports them (lib/ab, lib/prof); the product library does not
_TEST_SIGS = {
    "droid_conv_set_profile": ([_p], _i),
    "droid_alt_set_profile": ([_p], _i),
    "droid_alt_set_variant": ([_i], _i),
    "droid_alt_set_chunk": ([_i], _i),
    "droid_lookup_set_coop": ([_i], _i),
    "droid_conv_set_tile": ([_i], _i),
    "droid_conv_gate_tile": ([_i, _i, _i, _i], _i),
    "droid_chol_set_profile": ([_p], _i),
    "droid_chol_set_fault_inject": ([_i], _i),
}

EXPORTS = tuple(_SIGS)
TEST_EXPORTS = tuple(_TEST_SIGS)

for _name, (_args, _res) in _SIGS.items():
    if os.environ.get("DROID_HIP_LIB") and not hasattr(lib, _name):
        continue   # an older A/B build: entry points it predates stay unbound
    _fn = getattr(lib, _name)
    _fn.argtypes = _args
    _fn.restype = _res
for _name, (_args, _res) in _TEST_SIGS.items():
    if hasattr(lib, _name):
        _fn = getattr(lib, _name)
        _fn.argtypes = _args
        _fn.restype = _res
HAS_TESTING_HOOKS = all(hasattr(lib, _n) for _n in _TEST_SIGS)


def testing_hook(name):
    """A hook of include/droid_backends_testing.h, or a RuntimeError naming
    the build that has it (the product library exports none)."""
    if not hasattr(lib, name):
        raise RuntimeError("%s is a testing hook: only the A/B and profiling builds export it "
                           "(make -C droid-slam_amd/csrc ab prof; tests use the ab_backends fixture); "
                           "loaded library: %s" % (name, LIB_PATH))
    return getattr(lib, name)


def check(status, what):
    if status != 0:
        msg = lib.droid_last_error().decode("utf-8", "replace")
        raise RuntimeError("%s failed (status %d): %s" % (what, status, msg))
