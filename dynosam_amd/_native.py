"""Locate and load the in-tree native libraries.

libdynohip.so (HIP product path) and libdynosynth.so (host-only synthetic
graph generator) are built in-tree by __graft_entry__.build() into
dynosam_amd/lib/. There is no fallback: a missing library raises.
"""
import ctypes as C
import os

from . import _abi

# DYNOSAM_AMD_LIB_DIR points the loader at another build of the same
# libraries (kernel-variant A/B measurements); the default is the in-tree build
LIB_DIR = os.environ.get("DYNOSAM_AMD_LIB_DIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
_libs = {}


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path(name):
    return os.path.join(LIB_DIR, name)


def load(name):
    if name in _libs:
        return _libs[name]
    path = lib_path(name)
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = C.CDLL(path)
    _libs[name] = lib
    _declare(name, lib)
    return lib


def _declare(name, lib):
    P = C.POINTER
    if name == "libdynosynth.so":
        lib.dynosynth_config_default.argtypes = [P(_abi.SynthConfig)]
        lib.dynosynth_generate.argtypes = [P(_abi.SynthConfig), P(C.c_void_p)]
        lib.dynosynth_generate.restype = C.c_int
        lib.dynosynth_destroy.argtypes = [C.c_void_p]
        lib.dynosynth_graph.argtypes = [C.c_void_p, P(_abi.GraphView)]
        lib.dynosynth_num_values.argtypes = [C.c_void_p]
        lib.dynosynth_num_values.restype = C.c_size_t
        lib.dynosynth_values_len.argtypes = [C.c_void_p]
        lib.dynosynth_values_len.restype = C.c_size_t
        lib.dynosynth_value_keys.argtypes = [C.c_void_p]
        lib.dynosynth_value_keys.restype = P(C.c_uint64)
        lib.dynosynth_value_kinds.argtypes = [C.c_void_p]
        lib.dynosynth_value_kinds.restype = P(C.c_uint8)
        lib.dynosynth_value_data.argtypes = [C.c_void_p]
        lib.dynosynth_value_data.restype = P(C.c_double)
        lib.dynosynth_ground_truth.argtypes = [C.c_void_p]
        lib.dynosynth_ground_truth.restype = P(C.c_double)
    elif name == "libdynohip.so":
        vp = C.c_void_p
        lib.dynohip_abi_version.restype = C.c_int
        lib.dynohip_lm_params_default.argtypes = [P(_abi.LMParams)]
        lib.dynohip_create.argtypes = [C.c_int, P(vp)]
        lib.dynohip_create.restype = C.c_int
        lib.dynohip_destroy.argtypes = [vp]
        lib.dynohip_last_error.argtypes = [vp]
        lib.dynohip_last_error.restype = C.c_char_p
        lib.dynohip_set_graph.argtypes = [vp, P(_abi.GraphView)]
        lib.dynohip_set_graph.restype = C.c_int
        lib.dynohip_set_values.argtypes = [vp, P(C.c_uint64), P(C.c_uint8), P(C.c_double), C.c_size_t]
        lib.dynohip_set_values.restype = C.c_int
        lib.dynohip_get_values.argtypes = [vp, P(C.c_double), C.c_size_t]
        lib.dynohip_get_values.restype = C.c_int
        lib.dynohip_graph_error.argtypes = [vp, P(C.c_double)]
        lib.dynohip_graph_error.restype = C.c_int
        lib.dynohip_lm_reset.argtypes = [vp, P(_abi.LMParams)]
        lib.dynohip_lm_reset.restype = C.c_int
        lib.dynohip_iterate.argtypes = [vp, P(_abi.LMSummary)]
        lib.dynohip_iterate.restype = C.c_int
        lib.dynohip_optimize.argtypes = [vp, P(_abi.LMParams), P(_abi.LMSummary)]
        lib.dynohip_optimize.restype = C.c_int
        lib.dynohip_get_trace.argtypes = [vp, P(_abi.TraceEntry), C.c_size_t, P(C.c_size_t)]
        lib.dynohip_get_trace.restype = C.c_int
        lib.dynohip_solve_delta.argtypes = [vp, C.c_double, P(C.c_double), C.c_size_t, P(C.c_int)]
        lib.dynohip_solve_delta.restype = C.c_int
        lib.dynohip_pool_trim.argtypes = []
        lib.dynohip_pool_trim.restype = C.c_int
        lib.dynohip_linearize.argtypes = [vp, P(C.c_double), C.c_size_t]
        lib.dynohip_linearize.restype = C.c_int
        lib.dynohip_linearize_size.argtypes = [vp]
        lib.dynohip_linearize_size.restype = C.c_size_t
        lib.dynohip_values_snapshot.argtypes = [vp]
        lib.dynohip_values_snapshot.restype = C.c_int
        lib.dynohip_values_restore.argtypes = [vp]
        lib.dynohip_values_restore.restype = C.c_int
        lib.dynohip_get_stats.argtypes = [vp, P(_abi.Stats)]
        lib.dynohip_get_stats.restype = C.c_int
        lib.dynohip_set_timing.argtypes = [vp, C.c_int]
        lib.dynohip_set_timing.restype = C.c_int
        lib.dynohip_sliding_window_init.argtypes = [P(_abi.SlidingWindowState), C.c_int, C.c_int]
        lib.dynohip_sliding_window_init.restype = None
        lib.dynohip_sliding_window_check.argtypes = [P(_abi.SlidingWindowState), C.c_uint64, P(C.c_uint64), P(C.c_uint64)]
        lib.dynohip_sliding_window_check.restype = C.c_int
        lib.dynohip_set_exec_options.argtypes = [vp, C.c_int, C.c_int, C.c_int]
        lib.dynohip_set_exec_options.restype = C.c_int
        lib.dynohip_set_tile_ordering.argtypes = [C.c_int]
        lib.dynohip_set_tile_ordering.restype = None
        I32 = P(C.c_int32)
        lib.dynohip_plan_schedule.argtypes = [P(_abi.GraphView), P(C.c_uint64), P(C.c_uint8), C.c_size_t,
                                              P(_abi.ScheduleInfo)] + [I32] * 12
        lib.dynohip_plan_schedule.restype = C.c_int
        lib.dynohip_plan_export.argtypes = [P(_abi.GraphView), P(C.c_uint64), P(C.c_uint8), C.c_size_t, C.c_int,
                                            C.c_int, C.c_char_p, I32, C.c_size_t, P(C.c_size_t)]
        lib.dynohip_plan_export.restype = C.c_int
        lib.dynohip_set_partition.argtypes = [vp, C.c_int, C.c_int, _abi.ALLREDUCE_FN, vp]
        lib.dynohip_set_partition.restype = C.c_int
        lib.dynohip_value_owner.argtypes = [vp, I32, C.c_size_t, P(C.c_int64)]
        lib.dynohip_value_owner.restype = C.c_int
        lib.dynohip_full_batch_trigger.argtypes = [C.c_int64, C.c_uint64]
        lib.dynohip_full_batch_trigger.restype = C.c_int
        vp_ = C.c_void_p
        U64, I64, I32_, D, U8 = P(C.c_uint64), P(C.c_int64), P(C.c_int32), P(C.c_double), P(C.c_uint8)
        SZ = P(C.c_size_t)
        for fn, args, res in [
            ("dynob_map_create", [P(vp_)], C.c_int),
            ("dynob_map_destroy", [vp_], None),
            ("dynob_map_last_error", [vp_], C.c_char_p),
            ("dynob_map_update_observations", [vp_, vp_, C.c_size_t], C.c_int),
            ("dynob_map_update_sensor_pose", [vp_, C.c_uint64, D], C.c_int),
            ("dynob_map_update_object_motions", [vp_, C.c_uint64, I32_, D, C.c_size_t], C.c_int),
            ("dynob_map_query", [vp_, C.c_int, C.c_int64, C.c_int64, I64, C.c_size_t, SZ], C.c_int64),
            ("dynob_params_default", [P(_abi.BackendParams), C.c_int], None),
            ("dynob_formulation_create", [vp_, P(_abi.BackendParams), P(vp_)], C.c_int),
            ("dynob_formulation_destroy", [vp_], None),
            ("dynob_formulation_last_error", [vp_], C.c_char_p),
            ("dynob_set_initial_pose", [vp_, C.c_uint64, D], C.c_int),
            ("dynob_set_initial_pose_prior", [vp_, C.c_uint64, D], C.c_int),
            ("dynob_add_odometry", [vp_, C.c_uint64, D], C.c_int),
            ("dynob_update_static_observations", [vp_, C.c_uint64, C.c_int], C.c_int),
            ("dynob_update_dynamic_observations", [vp_, C.c_uint64, C.c_int], C.c_int),
            ("dynob_update_theta", [vp_, U64, U8, D, C.c_size_t], C.c_int),
            ("dynob_formulation_graph", [vp_, P(_abi.GraphView)], C.c_int),
            ("dynob_formulation_values", [vp_, P(U64), P(U8), P(D), SZ, SZ], C.c_int),
            ("dynob_formulation_factor_types", [vp_, U8, C.c_size_t, SZ], C.c_int),
            ("dynob_get_sensor_pose", [vp_, C.c_uint64, D], C.c_int),
            ("dynob_get_object_motions", [vp_, C.c_uint64, I32_, D, C.c_size_t, SZ], C.c_int),
            ("dynob_get_dynamic_landmarks", [vp_, C.c_uint64, I64, I32_, D, C.c_size_t, SZ], C.c_int),
            ("dynob_get_static_landmarks", [vp_, C.c_uint64, I64, D, C.c_size_t, SZ], C.c_int),
            ("dynob_object_centroid", [vp_, C.c_uint64, C.c_int32, D], C.c_int),
            ("dynob_post_update", [vp_], C.c_int),
            ("dynob_get_object_poses", [vp_, I32_, U64, D, C.c_size_t, SZ], C.c_int),
            ("dynob_log_backend_from_map", [vp_, C.c_char_p, C.c_char_p, C.c_int, C.c_int64, P(_abi.GroundTruth)],
             C.c_int),
            ("dynob_replay_open", [C.c_char_p, P(vp_)], C.c_int),
            ("dynob_replay_parse", [P(C.c_uint8), C.c_size_t, P(vp_)], C.c_int),
            ("dynob_replay_destroy", [vp_], None),
            ("dynob_replay_last_error", [vp_], C.c_char_p),
            ("dynob_replay_num_packets", [vp_], C.c_size_t),
            ("dynob_replay_packet", [vp_, C.c_size_t, P(_abi.InputPacket)], C.c_int),
            ("dynob_replay_ground_truth", [vp_, C.c_size_t, D, I32_, D, D, C.c_size_t, SZ], C.c_int),
            ("dynorefine_params_default", [P(_abi.RefineParams)], None),
            ("dynorefine_create", [C.c_int, P(vp_)], C.c_int),
            ("dynorefine_destroy", [vp_], None),
            ("dynorefine_last_error", [vp_], C.c_char_p),
            ("dynorefine_upload", [vp_, P(_abi.RefineBatch)], C.c_int),
            ("dynorefine_solve", [vp_, P(_abi.RefineParams), P(_abi.LMParams)], C.c_int),
            ("dynorefine_download", [vp_, D, U8, P(_abi.RefineResult)], C.c_int),
            ("dynorefine_run", [vp_, P(_abi.RefineBatch), P(_abi.RefineParams), P(_abi.LMParams), D, U8,
                                P(_abi.RefineResult)], C.c_int),
            ("dynorefine_last_solve_ms", [vp_], C.c_double),
            ("dynob_module_params_default", [P(_abi.ModuleParams)], None),
            ("dynob_module_create", [P(_abi.BackendParams), P(_abi.ModuleParams), P(vp_)], C.c_int),
            ("dynob_module_destroy", [vp_], None),
            ("dynob_module_last_error", [vp_], C.c_char_p),
            ("dynob_module_spin", [vp_, P(_abi.InputPacket), P(_abi.SpinResult)], C.c_int),
            ("dynob_module_flush", [vp_, P(_abi.SpinResult)], C.c_int),
            ("dynob_module_pending", [vp_], C.c_int),
            ("dynob_module_window_builds", [vp_, P(C.c_int), P(C.c_int)], C.c_int),
            ("dynob_module_map", [vp_], vp_),
            ("dynob_module_formulation", [vp_], vp_),
            ("dynob_module_last_problem", [vp_, P(_abi.GraphView), P(U64), P(U8), P(D), P(D), SZ, SZ], C.c_int),
            ("dynob_module_write_statistics", [vp_, C.c_char_p, C.c_char_p], C.c_int),
            ("dynob_module_statistics", [vp_, C.c_char_p, P(C.c_double), C.c_size_t, P(C.c_size_t)], C.c_int),
            ("dynob_module_statistics_labels", [vp_, C.c_char_p, C.c_size_t, P(C.c_size_t)], C.c_int),
        ]:
            f = getattr(lib, fn)
            f.argtypes = args
            f.restype = res
        for fn, args, res in [
            ("dynohip_symbol", [C.c_ubyte, C.c_uint64], C.c_uint64),
            ("dynohip_labeled_symbol", [C.c_ubyte, C.c_ubyte, C.c_uint64], C.c_uint64),
            ("dynohip_symbol_chr", [C.c_uint64], C.c_ubyte),
            ("dynohip_symbol_index", [C.c_uint64], C.c_uint64),
            ("dynohip_labeled_label", [C.c_uint64], C.c_ubyte),
            ("dynohip_labeled_index", [C.c_uint64], C.c_uint64),
            ("dynohip_cantor_pair", [C.c_uint64, C.c_uint64], C.c_uint64),
            ("dynohip_cantor_depair", [C.c_uint64, P(C.c_uint64), P(C.c_uint64)], None),
            ("dynohip_camera_pose_key", [C.c_uint64], C.c_uint64),
            ("dynohip_static_landmark_key", [C.c_int64], C.c_uint64),
            ("dynohip_dynamic_landmark_key", [C.c_uint64, C.c_int64, P(C.c_uint64)], C.c_int),
            ("dynohip_object_motion_key", [C.c_int, C.c_uint64], C.c_uint64),
            ("dynohip_object_pose_key", [C.c_int, C.c_uint64], C.c_uint64),
            ("dynohip_reconstruct_motion_info", [C.c_uint64, P(C.c_int), P(C.c_uint64)], C.c_int),
            ("dynohip_reconstruct_pose_info", [C.c_uint64, P(C.c_int), P(C.c_uint64)], C.c_int),
            ("dynohip_chr_extract", [C.c_uint64], C.c_ubyte),
        ]:
            f = getattr(lib, fn)
            f.argtypes = args
            f.restype = res
