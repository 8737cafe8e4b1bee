"""ctypes mirror of include/dynohip.h and include/dynosynth.h.

Plain struct layouts only; the product binding (dynosam_amd.optimizer) and
the test-only oracle binding (tests/oracle_binding.py) both use them.
"""
import ctypes as C

FACTOR_TYPES = (
    "pose_to_point",
    "landmark_motion_ternary",
    "between",
    "prior",
    "landmark_motion_pose",
    "landmark_pose_smoothing",
)
# keys per factor, residual dim, measurement dim, slot kinds (0 pose, 1 point)
FACTOR_NKEYS = (2, 3, 2, 1, 4, 3)
FACTOR_DIM = (3, 3, 6, 6, 3, 6)
FACTOR_MEAS = (3, 0, 12, 12, 0, 0)
FACTOR_SLOTS = ((0, 1), (1, 1, 0), (0, 0), (0,), (1, 1, 0, 0), (0, 0, 0))

POSE3 = 0
POINT3 = 1

# dynohip_allreduce_fn(void* ctx, double* buf, size_t n, int on_device, void* stream)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_size_t, C.c_int, C.c_void_p)


class FactorBlock(C.Structure):
    _fields_ = [
        ("n", C.c_size_t),
        ("keys", C.POINTER(C.c_uint64)),
        ("measured", C.POINTER(C.c_double)),
        ("sigmas", C.POINTER(C.c_double)),
        ("huber_k", C.POINTER(C.c_double)),
    ]


class GraphView(C.Structure):
    _fields_ = [(name, FactorBlock) for name in FACTOR_TYPES]


class LMParams(C.Structure):
    _fields_ = [
        ("lambda_initial", C.c_double),
        ("lambda_factor", C.c_double),
        ("lambda_upper_bound", C.c_double),
        ("lambda_lower_bound", C.c_double),
        ("min_model_fidelity", C.c_double),
        ("relative_error_tol", C.c_double),
        ("absolute_error_tol", C.c_double),
        ("error_tol", C.c_double),
        ("max_iterations", C.c_int),
        ("diagonal_damping", C.c_int),
        ("use_fixed_lambda_factor", C.c_int),
        ("reserved", C.c_int),
    ]

    @classmethod
    def gtsam_default(cls):
        """gtsam::LevenbergMarquardtParams() defaults (GTSAM 4.2.0)."""
        return cls(1e-5, 10.0, 1e5, 0.0, 1e-3, 1e-5, 1e-5, 0.0, 100, 0, 1, 0)


class LMSummary(C.Structure):
    _fields_ = [
        ("iterations", C.c_int),
        ("inner_iterations", C.c_int),
        ("initial_error", C.c_double),
        ("final_error", C.c_double),
        ("final_lambda", C.c_double),
        ("converged", C.c_int),
        ("reserved", C.c_int),
    ]


class TraceEntry(C.Structure):
    _fields_ = [
        ("outer_iteration", C.c_int),
        ("solved", C.c_int),
        ("accepted", C.c_int),
        ("stop", C.c_int),
        ("lambda_", C.c_double),
        ("current_error", C.c_double),
        ("new_error", C.c_double),
        ("old_linear_error", C.c_double),
        ("new_linear_error", C.c_double),
        ("model_fidelity", C.c_double),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("n_pose", C.c_int64),
        ("n_point", C.c_int64),
        ("n_factor", C.c_int64),
        ("n_chain", C.c_int64),
        ("n_edge", C.c_int64),
        ("reduced_dim", C.c_int64),
        ("tiles_stored", C.c_int64),
        ("band_max_tiles", C.c_int64),
        ("chol_levels", C.c_int64),
        ("back_levels", C.c_int64),
        ("nd_leaf", C.c_int64),
        ("lin_bytes", C.c_double),
        ("assembly_bytes", C.c_double),
        ("chol_flops", C.c_double),
        ("chol_tile_flops", C.c_double),
        ("ms_linearize", C.c_double),
        ("ms_schur", C.c_double),
        ("ms_assembly", C.c_double),
        ("ms_cholesky", C.c_double),
        ("ms_solve", C.c_double),
        ("ms_backsub", C.c_double),
        ("ms_retract_error", C.c_double),
        ("n_linearize", C.c_int64),
        ("n_solves", C.c_int64),
        ("lin_bytes_read", C.c_double),
        ("lin_bytes_impl", C.c_double),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class SlidingWindowState(C.Structure):
    _fields_ = [
        ("sliding_window", C.c_int),
        ("overlap_size", C.c_int),
        ("previous_trigger_frame", C.c_int),
        ("first_frame", C.c_int),
    ]


class SynthConfig(C.Structure):
    _fields_ = [
        ("frames", C.c_int),
        ("objects", C.c_int),
        ("static_landmarks", C.c_int),
        ("dyn_slots", C.c_int),
        ("static_track_len", C.c_int),
        ("dyn_track_len", C.c_int),
        ("seed", C.c_uint64),
        ("noise_code_defaults", C.c_int),
        ("object_visible_frames", C.c_int),
        ("formulation", C.c_int),
        ("smoothing", C.c_int),
        ("robust", C.c_int),
    ]


def trace_to_dicts(entries):
    out = []
    for e in entries:
        out.append(
            dict(
                outer_iteration=e.outer_iteration,
                solved=e.solved,
                accepted=e.accepted,
                stop=e.stop,
                lam=e.lambda_,
                current_error=e.current_error,
                new_error=e.new_error,
                old_linear_error=e.old_linear_error,
                new_linear_error=e.new_linear_error,
                model_fidelity=e.model_fidelity,
            )
        )
    return out


class ScheduleInfo(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("n_pose", "n_tiles", "n_slots", "n_ftask", "n_pairs", "n_flevel", "n_btask",
                                          "n_blevel", "n_bent", "n_red_blocks", "nd_leaf")]


# ---- include/dynobackend.h -------------------------------------------------
class Measurement(C.Structure):
    """dynob_measurement: one tracked landmark measurement (camera frame)."""
    _fields_ = [
        ("tracklet_id", C.c_int64),
        ("object_id", C.c_int32),
        ("reserved", C.c_int32),
        ("frame_id", C.c_uint64),
        ("landmark", C.c_double * 3),
    ]


MEASUREMENT_DTYPE = None  # numpy structured dtype with the same layout (set lazily by backend.py)


class BackendParams(C.Structure):
    _fields_ = [
        ("formulation", C.c_int),
        ("min_static_observations", C.c_int),
        ("min_dynamic_observations", C.c_int),
        ("use_smoothing_factor", C.c_int),
        ("init_H_with_identity", C.c_int),
        ("use_robust_kernels", C.c_int),
        ("k_huber_3d_points", C.c_double),
        ("static_point_sigma", C.c_double),
        ("dynamic_point_sigma", C.c_double),
        ("motion_ternary_sigma", C.c_double),
        ("odometry_sigmas", C.c_double * 6),
        ("smoothing_sigmas", C.c_double * 6),
        ("initial_pose_prior_sigma", C.c_double),
    ]


class InputPacket(C.Structure):
    _fields_ = [
        ("frame_id", C.c_uint64),
        ("timestamp", C.c_double),
        ("T_world_camera", C.c_double * 12),
        ("static_measurements", C.c_void_p),
        ("n_static", C.c_size_t),
        ("dynamic_measurements", C.c_void_p),
        ("n_dynamic", C.c_size_t),
        ("motion_object_ids", C.POINTER(C.c_int32)),
        ("motions12", C.POINTER(C.c_double)),
        ("n_motions", C.c_size_t),
    ]


class ModuleParams(C.Structure):
    _fields_ = [
        ("use_full_batch_opt", C.c_int),
        ("full_batch_frame", C.c_int64),
        ("opt_window_size", C.c_int),
        ("opt_window_overlap", C.c_int),
        ("optimize", C.c_int),
        ("device_id", C.c_int),
        ("post_update", C.c_int),
        ("windows_in_flight", C.c_int),
        ("lm", LMParams),
    ]


class SpinResult(C.Structure):
    _fields_ = [
        ("optimized", C.c_int),
        ("iterations", C.c_int),
        ("inner_iterations", C.c_int),
        ("windows_merged", C.c_int),
        ("window_start", C.c_uint64),
        ("window_end", C.c_uint64),
        ("error_before", C.c_double),
        ("error_after", C.c_double),
        ("ms_construct", C.c_double),
        ("ms_optimize", C.c_double),
    ]


class GroundTruth(C.Structure):
    """dynob_ground_truth"""
    _fields_ = [
        ("n_frames", C.c_size_t),
        ("frame_ids", C.POINTER(C.c_uint64)),
        ("X_world12", C.POINTER(C.c_double)),
        ("n_objects", C.c_size_t),
        ("object_frame_ids", C.POINTER(C.c_uint64)),
        ("object_ids", C.POINTER(C.c_int32)),
        ("L_world12", C.POINTER(C.c_double)),
        ("prev_H_current_world12", C.POINTER(C.c_double)),
    ]


# ---- include/dynorefine.h --------------------------------------------------
class RefineBatch(C.Structure):
    _fields_ = [
        ("n_problems", C.c_size_t),
        ("track_start", C.POINTER(C.c_int32)),
        ("X_k_1", C.POINTER(C.c_double)),
        ("X_k", C.POINTER(C.c_double)),
        ("H_init", C.POINTER(C.c_double)),
        ("calibration", C.POINTER(C.c_double)),
        ("kp_k_1", C.POINTER(C.c_double)),
        ("kp_k", C.POINTER(C.c_double)),
        ("m_k_1", C.POINTER(C.c_double)),
        ("m_k", C.POINTER(C.c_double)),
        ("X_k_1_init", C.POINTER(C.c_double)),
        ("X_k_init", C.POINTER(C.c_double)),
        ("ternary_inactive", C.POINTER(C.c_uint8)),
    ]


class RefineParams(C.Structure):
    _fields_ = [
        ("landmark_motion_sigma", C.c_double),
        ("projection_sigma", C.c_double),
        ("k_huber", C.c_double),
        ("prior_sigma", C.c_double),
        ("outlier_reject", C.c_int),
        ("reserved", C.c_int),
    ]


class RefineResult(C.Structure):
    _fields_ = [
        ("iterations", C.c_int),
        ("inner_iterations", C.c_int),
        ("status", C.c_int),
        ("n_outliers", C.c_int),
        ("error_before", C.c_double),
        ("error_after", C.c_double),
    ]
