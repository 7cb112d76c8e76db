"""ctypes binding of the mi_ba C-ABI (include/mi_ba.h) and the synthetic
scene tool (include/mi_ba_synthetic.h).

This is plumbing for tests/ and bench.py: the product is libmi_ba.so (HIP
kernels + C++ runtime).  Loading the library never falls back to anything:
if libmi_ba.so is missing, `load()` raises; on a machine without an MI355X
the compute entry points return MI_BA_ERR_NO_DEVICE.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MI_BA_LIB=ab selects the tools-only A/B build (libmi_ba_ab.so: `make ab`,
# the measured-slower kernel variants compiled in) for tools/ab_*.py; tests,
# smoke() and bench.py load the product library.
AB_LIB_PATH = os.path.join(_HERE, "libmi_ba_ab.so")
LIB_PATH = AB_LIB_PATH if os.environ.get("MI_BA_LIB") == "ab" else os.path.join(_HERE, "libmi_ba.so")
SYNTH_PATH = os.path.join(_HERE, "libmi_ba_synth.so")

# status codes / enums (mi_ba.h)
OK, ERR_INVALID_ARGUMENT, ERR_NO_DEVICE, ERR_UNSUPPORTED, ERR_HIP, ERR_NO_RESIDUALS, ERR_STATE, ERR_OOM = range(8)
SIMPLE_PINHOLE, PINHOLE, SIMPLE_RADIAL, RADIAL, OPENCV = range(5)
LOSS_TRIVIAL, LOSS_SOFT_L1, LOSS_CAUCHY = range(3)
SOLVER_AUTO, SOLVER_DENSE_SCHUR, SOLVER_ITERATIVE_SCHUR = range(3)
CONVERGENCE, NO_CONVERGENCE, FAILURE, USER_SUCCESS, USER_FAILURE = range(5)
SOLVER_CONTINUE, SOLVER_ABORT, SOLVER_TERMINATE_SUCCESSFULLY = range(3)
CYLINDER_DEFAULT, CYLINDER_BY_2_POINTS = range(2)
OUT_OF_BOUNDS, INVALID_DEPTH, VALID = -1, -2, 10
NUM_PARAMS = {SIMPLE_PINHOLE: 3, PINHOLE: 4, SIMPLE_RADIAL: 4, RADIAL: 5, OPENCV: 8}
MODEL_NAMES = {"SIMPLE_PINHOLE": 0, "PINHOLE": 1, "SIMPLE_RADIAL": 2, "RADIAL": 3, "OPENCV": 4}

_dp = C.POINTER(C.c_double)
_fp = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_u8p = C.POINTER(C.c_uint8)


class IterationSummary(C.Structure):
    """mi_ba_iteration_summary (ceres::IterationSummary fields)."""
    _fields_ = [
        ("iteration", C.c_int32),
        ("step_is_valid", C.c_int32),
        ("step_is_successful", C.c_int32),
        ("linear_solver_iterations", C.c_int32),
        ("cost", C.c_double),
        ("cost_change", C.c_double),
        ("relative_decrease", C.c_double),
        ("trust_region_radius", C.c_double),
        ("step_norm", C.c_double),
        ("iteration_time_in_seconds", C.c_double),
        ("cumulative_time_in_seconds", C.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# mi_ba_iteration_callback_fn: int32 (void* user, const mi_ba_iteration_summary*)
ITERATION_CALLBACK_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.POINTER(IterationSummary))


class Options(C.Structure):
    _fields_ = [
        ("loss_function_type", C.c_int32),
        ("loss_function_scale", C.c_double),
        ("refine_focal_length", C.c_int32),
        ("refine_principal_point", C.c_int32),
        ("refine_extra_params", C.c_int32),
        ("refine_extrinsics", C.c_int32),
        ("print_summary", C.c_int32),
        ("max_num_iterations", C.c_int32),
        ("function_tolerance", C.c_double),
        ("gradient_tolerance", C.c_double),
        ("parameter_tolerance", C.c_double),
        ("max_linear_solver_iterations", C.c_int32),
        ("max_num_consecutive_invalid_steps", C.c_int32),
        ("linear_solver_type", C.c_int32),
        ("eta", C.c_double),
        ("initial_trust_region_radius", C.c_double),
        ("min_relative_decrease", C.c_double),
        ("device", C.c_int32),
        ("semantic_weight", C.c_double),
        ("iteration_callback", ITERATION_CALLBACK_FN),
        ("callback_user", C.c_void_p),
        ("update_state_every_iteration", C.c_int32),
        ("stop_flag", _i32p),
    ]

    def set_callback(self, fn, update_state_every_iteration: bool = False):
        """Install `fn(IterationSummary) -> MI_BA_SOLVER_*` (None / a falsy
        return continues) as the solver's iteration callback; the thunk is
        kept alive on the options object."""
        def _cb(_user, summary):
            try:
                r = fn(summary.contents)
                return int(r) if r else SOLVER_CONTINUE
            except Exception:  # noqa: BLE001 — an exception in the callback aborts the solve
                return SOLVER_ABORT
        self._thunk = ITERATION_CALLBACK_FN(_cb)
        self.iteration_callback = self._thunk
        self.update_state_every_iteration = 1 if update_state_every_iteration else 0
        return self

    def set_stop_flag(self, flag: "np.ndarray"):
        """Point the solver's stop flag at flag[0] (an int32 numpy array the
        caller keeps alive and may set from another thread)."""
        assert flag.dtype == np.int32 and flag.flags.c_contiguous
        self._stop = flag
        self.stop_flag = flag.ctypes.data_as(_i32p)
        return self


class Problem(C.Structure):
    _fields_ = [
        ("camera_model", C.c_int32),
        ("num_cameras", C.c_int32),
        ("camera_params", _dp),
        ("camera_constant", _u8p),
        ("num_images", C.c_int32),
        ("qvec", _dp),
        ("tvec", _dp),
        ("image_camera", _i32p),
        ("image_in_config", _u8p),
        ("image_constant_pose", _u8p),
        ("image_constant_tvec", _u8p),
        ("num_points", C.c_int64),
        ("xyz", _dp),
        ("point_config", _u8p),
        ("num_obs", C.c_int64),
        ("obs_xy", _dp),
        ("obs_image", _i32p),
        ("obs_point", _i32p),
        ("camera_model_ids", _i32p),
    ]


class Cylinder(C.Structure):
    _fields_ = [("qvec", C.c_double * 4), ("tvec", C.c_double * 3), ("radius", C.c_double), ("height", C.c_double)]


class Gsba(C.Structure):
    _fields_ = [
        ("height", C.c_int32),
        ("width", C.c_int32),
        ("trunk_mask", _u8p),
        ("num_cylinders", C.c_int32),
        ("cylinders", C.POINTER(Cylinder)),
        ("refine_geometry", C.c_int32),
        ("numeric_relative_step_size", C.c_double),
        ("include_landmark_error", C.c_int32),
        ("landmark_error_weight", C.c_double),
        ("cylinder_parametrization", C.c_int32),
        ("image_height", _i32p),
        ("image_width", _i32p),
    ]


class Semantic(C.Structure):
    _fields_ = [
        ("height", C.c_int32),
        ("width", C.c_int32),
        ("depth", _fp),
        ("label", _fp),
        ("num_pairs", C.c_int32),
        ("pairs", _i32p),
        ("pixel_step", C.c_int32),
        ("depth_error_threshold", C.c_double),
        ("numeric_relative_step_size", C.c_double),
        ("image_height", _i32p),
        ("image_width", _i32p),
    ]


def _planes(maps, dtype):
    """[I][H][W] array -> (it, None, None); list of per-image [H_i][W_i]
    arrays (ABI 4: each image its own size) -> (planes back to back, heights,
    widths)."""
    if isinstance(maps, np.ndarray):
        return np.ascontiguousarray(maps, dtype), None, None
    hs = np.array([np.shape(m)[0] if np.ndim(m) == 2 else 0 for m in maps], np.int32)
    ws = np.array([np.shape(m)[1] if np.ndim(m) == 2 else 0 for m in maps], np.int32)
    flat = [np.ascontiguousarray(m, dtype).ravel() for m in maps]
    return (np.concatenate(flat) if flat else np.zeros(0, dtype)), hs, ws


class Summary(C.Structure):
    _fields_ = [
        ("num_residuals_reduced", C.c_int64),
        ("num_effective_parameters_reduced", C.c_int64),
        ("num_successful_steps", C.c_int32),
        ("num_unsuccessful_steps", C.c_int32),
        ("termination_type", C.c_int32),
        ("initial_cost", C.c_double),
        ("final_cost", C.c_double),
        ("fixed_cost", C.c_double),
        ("total_time_in_seconds", C.c_double),
        ("jacobian_evaluation_time_in_seconds", C.c_double),
        ("num_jacobian_evaluations", C.c_int32),
        ("num_linear_solver_iterations", C.c_int32),
        ("num_semantic_residuals", C.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class SetupInfo(C.Structure):
    _fields_ = [
        ("num_residual_blocks", C.c_int64),
        ("num_residuals_reduced", C.c_int64),
        ("num_effective_parameters_reduced", C.c_int64),
        ("num_variable_images", C.c_int64),
        ("num_variable_cameras", C.c_int64),
        ("num_variable_points", C.c_int64),
        ("camera_tangent_size", C.c_int32),
    ]


class SynthConfig(C.Structure):
    _fields_ = [
        ("camera_model", C.c_int32),
        ("num_images", C.c_int32),
        ("num_points", C.c_int64),
        ("track_length", C.c_int32),
        ("image_size", C.c_int32),
        ("focal_factor", C.c_double),
        ("extra", C.c_double * 4),
        ("rotation_range", C.c_double),
        ("noise", C.c_double),
        ("seed", C.c_uint32),
    ]


def _ptr(a, t):
    return None if a is None else a.ctypes.data_as(t)


_lib = None
_synth = None
# mi_ba_host_allreduce_fn: int32 (double* data, int64 n, void* user)
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int32, _dp, C.c_int64, C.c_void_p)
COMM_ID_BYTES = 128


def load(path: str = LIB_PATH):
    """Load libmi_ba.so; raises if the product library is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{os.path.basename(path)} not built at {path} "
                           "(run __graft_entry__.build(); the A/B build: make -C semantic-bundle-adjustment-colmap_amd ab)")
    lib = C.CDLL(path)
    lib.mi_ba_abi_version.restype = C.c_int32
    lib.mi_ba_status_string.restype = C.c_char_p
    lib.mi_ba_status_string.argtypes = [C.c_int32]
    lib.mi_ba_num_params.restype = C.c_int32
    lib.mi_ba_num_params.argtypes = [C.c_int32]
    lib.mi_ba_device_count.argtypes = [_i32p]
    lib.mi_ba_default_options.argtypes = [C.POINTER(Options)]
    lib.mi_ba_default_options.restype = None
    lib.mi_ba_setup_stats.argtypes = [C.POINTER(Options), C.POINTER(Problem), C.POINTER(SetupInfo)]
    lib.mi_ba_solve.argtypes = [C.POINTER(Options), C.POINTER(Problem), C.POINTER(Semantic), C.POINTER(Summary)]
    lib.mi_ba_context_create.argtypes = [C.POINTER(Options), C.POINTER(Problem), C.POINTER(Semantic),
                                         C.POINTER(C.c_void_p)]
    lib.mi_ba_context_destroy.argtypes = [C.c_void_p]
    lib.mi_ba_context_destroy.restype = None
    for name in ("mi_ba_linearize", "mi_ba_evaluate_jacobian", "mi_ba_evaluate_semantic", "mi_ba_synchronize",
                 "mi_ba_reset_kernel_times"):
        getattr(lib, name).argtypes = [C.c_void_p]
    lib.mi_ba_context_dims.argtypes = [C.c_void_p, _i64p, _i32p, _i64p]
    lib.mi_ba_download_jacobian.argtypes = [C.c_void_p, _i64p, _dp, _dp]
    lib.mi_ba_download_semantic.argtypes = [C.c_void_p, _i32p, _i32p, _dp, _dp]
    lib.mi_ba_semantic_export.argtypes = [C.c_void_p, C.c_int32, C.c_int32, _i64p, _i32p, _i32p, _dp, _dp]
    lib.mi_ba_context_cost.argtypes = [C.c_void_p, _dp]
    lib.mi_ba_context_solve.argtypes = [C.c_void_p, C.POINTER(Summary)]
    lib.mi_ba_context_writeback.argtypes = [C.c_void_p]
    lib.mi_ba_set_timing.argtypes = [C.c_void_p, C.c_int32]
    lib.mi_ba_set_tuning.argtypes = [C.c_void_p, C.c_char_p, C.c_int32]
    lib.mi_ba_kernel_time.argtypes = [C.c_void_p, C.c_char_p, _dp, _i64p]
    lib.mi_ba_comm_unique_id.argtypes = [C.c_char_p]
    lib.mi_ba_context_set_comm.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_char_p]
    lib.mi_ba_comm_pending_setups.argtypes = []
    lib.mi_ba_comm_pending_setups.restype = C.c_int32
    lib.mi_ba_context_set_host_reducer.argtypes = [C.c_void_p, C.c_int32, C.c_int32, HOST_ALLREDUCE_FN, C.c_void_p]
    lib.mi_ba_dense_cholesky.argtypes = [C.c_int32, C.c_int32, _dp, _dp, C.c_int32, C.c_int32, C.c_int32, _i32p]
    lib.mi_ba_dense_cholesky_ex.argtypes = [C.c_int32, C.c_int32, _dp, _dp, C.c_int32, C.c_int32, C.c_int32,
                                            C.c_int32, _i32p]
    lib.mi_ba_gsba_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.mi_ba_gsba_evaluate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64),
                                        C.c_void_p, C.c_void_p, C.c_void_p]
    lib.mi_ba_solve_in.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.mi_ba_solve_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                      C.c_void_p]
    lib.mi_ba_squared_reprojection_errors.argtypes = [C.c_void_p, C.c_int32, _dp]
    lib.mi_ba_filter_points3d.argtypes = [C.c_void_p, C.c_double, _u8p, C.c_int32, _u8p, _u8p, _dp,
                                          C.POINTER(C.c_int64)]
    lib.mi_ba_positive_depth.argtypes = [C.c_void_p, _u8p, C.c_int32, _u8p, C.POINTER(C.c_int64)]
    _lib = lib
    return lib


def ab_build() -> bool:
    """True when the loaded library is the tools-only A/B build."""
    load()
    return LIB_PATH == AB_LIB_PATH


def load_synth(path: str = SYNTH_PATH):
    global _synth
    if _synth is not None:
        return _synth
    lib = C.CDLL(path)
    lib.mi_ba_synth_num_obs.restype = C.c_int64
    lib.mi_ba_synth_num_obs.argtypes = [C.POINTER(SynthConfig)]
    lib.mi_ba_synth_generate.argtypes = [C.POINTER(SynthConfig), _dp, _dp, _dp, _i32p, _dp, _dp, _i32p, _i32p]
    lib.mi_ba_synth_render.argtypes = [C.c_int32, C.c_int32, _dp, _dp, _dp, _i32p, C.c_int32, C.c_int32,
                                       C.c_double, C.c_double, _fp, _fp]
    _synth = lib
    return lib


class MiBaError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = _lib.mi_ba_status_string(status).decode() if _lib else str(status)
        super().__init__(f"{what}: mi_ba status {status} ({msg})")


def check(status: int, what: str = ""):
    if status != OK:
        raise MiBaError(status, what)


def default_options(**kw) -> Options:
    o = Options()
    load().mi_ba_default_options(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise AttributeError(k)
        setattr(o, k, v)
    return o


@dataclass
class Scene:
    """Flattened Reconstruction + BundleAdjustmentConfig (numpy-owned)."""
    camera_model: int
    camera_params: np.ndarray            # [C][np] f64 (one model), or packed per camera (camera_models)
    qvec: np.ndarray                     # [I][4]
    tvec: np.ndarray                     # [I][3]
    image_camera: np.ndarray             # [I] i32
    xyz: np.ndarray                      # [P][3]
    obs_xy: np.ndarray                   # [N][2]
    obs_image: np.ndarray                # [N] i32
    obs_point: np.ndarray                # [N] i32
    camera_constant: Optional[np.ndarray] = None
    image_in_config: Optional[np.ndarray] = None
    image_constant_pose: Optional[np.ndarray] = None
    image_constant_tvec: Optional[np.ndarray] = None
    point_config: Optional[np.ndarray] = None
    camera_models: Optional[np.ndarray] = None  # [C] i32 model id per camera (mixed models)
    _keep: list = field(default_factory=list, repr=False)

    @property
    def num_cameras(self):
        return int(len(self.camera_models)) if self.camera_models is not None else int(self.camera_params.shape[0])

    def camera_param_offsets(self):
        """Offset of each camera's params in the flattened camera_params (+ total)."""
        if self.camera_models is None:
            n = NUM_PARAMS[self.camera_model]
            return np.arange(self.num_cameras + 1, dtype=np.int64) * n
        return np.concatenate([[0], np.cumsum([NUM_PARAMS[int(m)] for m in self.camera_models])]).astype(np.int64)

    @property
    def num_images(self):
        return int(self.qvec.shape[0])

    @property
    def num_points(self):
        return int(self.xyz.shape[0])

    @property
    def num_obs(self):
        return int(self.obs_image.shape[0])

    def copy(self) -> "Scene":
        def c(a):
            return None if a is None else a.copy()
        return Scene(self.camera_model, c(self.camera_params), c(self.qvec), c(self.tvec), c(self.image_camera),
                     c(self.xyz), c(self.obs_xy), c(self.obs_image), c(self.obs_point), c(self.camera_constant),
                     c(self.image_in_config), c(self.image_constant_pose), c(self.image_constant_tvec),
                     c(self.point_config), c(self.camera_models))

    def gauge(self, const_pose=0, const_tvec_image=1, const_tvec_mask=1):
        """BundleAdjustmentController gauge (controllers/bundle_adjustment.cc:94-95)."""
        I = self.num_images
        self.image_constant_pose = np.zeros(I, np.uint8)
        self.image_constant_pose[const_pose] = 1
        self.image_constant_tvec = np.zeros(I, np.uint8)
        if const_tvec_image is not None and const_tvec_image < I:
            self.image_constant_tvec[const_tvec_image] = const_tvec_mask
        return self

    def _normalize(self):
        for name, dt in (("camera_params", np.float64), ("qvec", np.float64), ("tvec", np.float64),
                         ("xyz", np.float64), ("obs_xy", np.float64), ("image_camera", np.int32),
                         ("obs_image", np.int32), ("obs_point", np.int32)):
            a = getattr(self, name)
            if a.dtype != dt or not a.flags.c_contiguous:
                setattr(self, name, np.ascontiguousarray(a, dtype=dt))
        if self.camera_models is not None and (self.camera_models.dtype != np.int32
                                               or not self.camera_models.flags.c_contiguous):
            self.camera_models = np.ascontiguousarray(self.camera_models, dtype=np.int32)
        for name in ("camera_constant", "image_in_config", "image_constant_pose", "image_constant_tvec",
                     "point_config"):
            a = getattr(self, name)
            if a is not None and (a.dtype != np.uint8 or not a.flags.c_contiguous):
                setattr(self, name, np.ascontiguousarray(a, dtype=np.uint8))

    def problem(self) -> Problem:
        self._normalize()
        p = Problem()
        p.camera_model = self.camera_model
        p.num_cameras = self.num_cameras
        p.camera_params = _ptr(self.camera_params, _dp)
        p.camera_model_ids = _ptr(self.camera_models, _i32p)
        p.camera_constant = _ptr(self.camera_constant, _u8p)
        p.num_images = self.num_images
        p.qvec = _ptr(self.qvec, _dp)
        p.tvec = _ptr(self.tvec, _dp)
        p.image_camera = _ptr(self.image_camera, _i32p)
        p.image_in_config = _ptr(self.image_in_config, _u8p)
        p.image_constant_pose = _ptr(self.image_constant_pose, _u8p)
        p.image_constant_tvec = _ptr(self.image_constant_tvec, _u8p)
        p.num_points = self.num_points
        p.xyz = _ptr(self.xyz, _dp)
        p.point_config = _ptr(self.point_config, _u8p)
        p.num_obs = self.num_obs
        p.obs_xy = _ptr(self.obs_xy, _dp)
        p.obs_image = _ptr(self.obs_image, _i32p)
        p.obs_point = _ptr(self.obs_point, _i32p)
        return p


@dataclass
class SemanticInput:
    depth: object              # [I][H][W] f32, or a list of per-image [H_i][W_i] maps
    label: object              # as depth
    pairs: np.ndarray          # [K][2] i32
    pixel_step: int = 10
    depth_error_threshold: float = 2.0
    numeric_relative_step_size: float = 1e-3

    def struct(self) -> Semantic:
        self._depth, self._h, self._w = _planes(self.depth, np.float32)
        self._label, hl, wl = _planes(self.label, np.float32)
        if (self._h is None) != (hl is None) or (self._h is not None and
                                                  (not np.array_equal(self._h, hl) or not np.array_equal(self._w, wl))):
            raise ValueError("depth and label maps differ in size")
        self.pairs = np.ascontiguousarray(self.pairs, np.int32).reshape(-1, 2)
        s = Semantic()
        if self._h is None:
            s.height = self._depth.shape[1]
            s.width = self._depth.shape[2]
        else:
            s.height = s.width = 0
            s.image_height = _ptr(self._h, _i32p)
            s.image_width = _ptr(self._w, _i32p)
        s.depth = _ptr(self._depth, _fp)
        s.label = _ptr(self._label, _fp)
        s.num_pairs = self.pairs.shape[0]
        s.pairs = _ptr(self.pairs, _i32p)
        s.pixel_step = self.pixel_step
        s.depth_error_threshold = self.depth_error_threshold
        s.numeric_relative_step_size = self.numeric_relative_step_size
        return s


def comm_pending_setups() -> int:
    """Communicator set-ups still running on their helper threads."""
    return int(load().mi_ba_comm_pending_setups())


def comm_unique_id() -> bytes:
    """RCCL unique id for mi_ba_context_set_comm (create on rank 0, broadcast)."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    check(load().mi_ba_comm_unique_id(buf), "mi_ba_comm_unique_id")
    return buf.raw


def shard_scene(scene: "Scene", rank: int, world: int, semantic: Optional["SemanticInput"] = None):
    """Rank `rank`'s shard for the multi-rank LM: every camera and image, the
    observations of the points in the rank's contiguous point range, and the
    rank's contiguous range of semantic image pairs."""
    P = scene.num_points
    p0, p1 = P * rank // world, P * (rank + 1) // world
    m = (scene.obs_point >= p0) & (scene.obs_point < p1)
    sh = scene.copy()
    sh.obs_xy, sh.obs_image, sh.obs_point = scene.obs_xy[m].copy(), scene.obs_image[m].copy(), scene.obs_point[m].copy()
    sem = None
    if semantic is not None:
        K = len(semantic.pairs)
        sem = SemanticInput(semantic.depth, semantic.label, np.asarray(semantic.pairs)[K * rank // world:K * (rank + 1) // world],
                            semantic.pixel_step, semantic.depth_error_threshold, semantic.numeric_relative_step_size)
    return sh, sem


def dense_cholesky(A: np.ndarray, b: Optional[np.ndarray] = None, device: int = 0, panel: int = 512,
                   lookahead: int = 1, own_diag: int = 6, solve: int = 2):
    """mi_ba_dense_cholesky: the reduced-camera-system factorisation on a
    caller-supplied SPD matrix.  Returns (L, x, info): L lower triangular
    (strict upper zeroed), x the solution of A x = b (None without b)."""
    n = A.shape[0]
    F = np.asfortranarray(A, dtype=np.float64).copy(order="F")
    x = None if b is None else np.ascontiguousarray(b, dtype=np.float64).copy()
    info = C.c_int32(0)
    check(load().mi_ba_dense_cholesky_ex(device, n, F.ctypes.data_as(_dp), _ptr(x, _dp), panel, lookahead, own_diag,
                                         solve, C.byref(info)), "mi_ba_dense_cholesky_ex")
    return np.tril(F), x, info.value


@dataclass
class GsbaInput:
    """mi_ba_gsba: trunk masks [I][H][W] (uint8, 1 = trunk class) and
    cylinders [N][9] = q(4) t(3) radius height (updated in place by solves)."""
    masks: np.ndarray
    cylinders: np.ndarray
    refine_geometry: int = 1
    numeric_relative_step_size: float = 1e-3
    include_landmark_error: int = 0
    landmark_error_weight: float = 1.0
    cylinder_parametrization: int = CYLINDER_DEFAULT

    def copy(self) -> "GsbaInput":
        return GsbaInput(self.masks, self.cylinders.copy(), self.refine_geometry, self.numeric_relative_step_size,
                         self.include_landmark_error, self.landmark_error_weight, self.cylinder_parametrization)

    def struct(self):
        self._masks, self._h, self._w = _planes(self.masks, np.uint8)
        n = len(self.cylinders)
        arr = (Cylinder * max(1, n))()
        for k in range(n):
            c = self.cylinders[k]
            arr[k].qvec[:] = list(c[:4])
            arr[k].tvec[:] = list(c[4:7])
            arr[k].radius = float(c[7])
            arr[k].height = float(c[8])
        g = Gsba()
        if self._h is None:
            g.height, g.width = int(self._masks.shape[1]), int(self._masks.shape[2])
        else:
            g.height = g.width = 0
            g.image_height = _ptr(self._h, _i32p)
            g.image_width = _ptr(self._w, _i32p)
        g.trunk_mask = _ptr(self._masks, _u8p)
        g.num_cylinders = n
        g.cylinders = C.cast(arr, C.POINTER(Cylinder))
        g.refine_geometry = self.refine_geometry
        g.numeric_relative_step_size = self.numeric_relative_step_size
        g.include_landmark_error = self.include_landmark_error
        g.landmark_error_weight = self.landmark_error_weight
        g.cylinder_parametrization = self.cylinder_parametrization
        return g, arr

    def read_back(self, arr):
        for k in range(len(self.cylinders)):
            self.cylinders[k, :4] = list(arr[k].qvec)
            self.cylinders[k, 4:7] = list(arr[k].tvec)
            self.cylinders[k, 7] = arr[k].radius
            self.cylinders[k, 8] = arr[k].height


def gsba_solve(options: Options, scene: Scene, gsba: GsbaInput) -> Summary:
    """GeometricSemanticBundleAdjuster<Cylinder>::Solve on the device."""
    s = Summary()
    p = scene.problem()
    g, arr = gsba.struct()
    check(load().mi_ba_gsba_solve(C.byref(options), C.byref(p), C.byref(g), C.byref(s)), "mi_ba_gsba_solve")
    gsba.read_back(arr)
    return s


def gsba_evaluate(options: Options, scene: Scene, gsba: GsbaInput):
    """Every GSBA block: (ids [n][2], residual 1 - IoU [n], ambient J [n][16])."""
    p = scene.problem()
    g, arr = gsba.struct()
    n = C.c_int64(0)
    lib = load()
    check(lib.mi_ba_gsba_evaluate(C.byref(options), C.byref(p), C.byref(g), 0, C.byref(n), None, None, None),
          "mi_ba_gsba_evaluate")
    ids = np.zeros((n.value, 2), np.int32)
    r = np.zeros(n.value)
    J = np.zeros((n.value, 16))
    check(lib.mi_ba_gsba_evaluate(C.byref(options), C.byref(p), C.byref(g), n.value, C.byref(n),
                                  ids.ctypes.data_as(C.c_void_p), r.ctypes.data_as(C.c_void_p),
                                  J.ctypes.data_as(C.c_void_p)), "mi_ba_gsba_evaluate")
    return ids, r, J


def look_at_qvec(center, target):
    """World->camera (qvec, tvec) of a camera at `center` looking at `target`
    (image x right, y down, z forward; world z up)."""
    z = np.asarray(target, float) - np.asarray(center, float)
    z /= np.linalg.norm(z)
    x = np.cross(z, [0.0, 0.0, 1.0])
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z])
    t = -R @ np.asarray(center, float)
    # rotation matrix -> (w, x, y, z)
    w = np.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2.0
    if w > 1e-6:
        q = np.array([w, (R[2, 1] - R[1, 2]) / (4 * w), (R[0, 2] - R[2, 0]) / (4 * w), (R[1, 0] - R[0, 1]) / (4 * w)])
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k]) * 2.0
        q = np.zeros(4)
        q[0] = (R[k, j] - R[j, k]) / s
        q[1 + i] = 0.25 * s
        q[1 + j] = (R[j, i] + R[i, j]) / s
        q[1 + k] = (R[k, i] + R[i, k]) / s
    return q / np.linalg.norm(q), t


def gsba_scene(num_images=10, num_cylinders=5, height=240, width=320, seed=0, points=0):
    """Synthetic GSBA workload: SIMPLE_PINHOLE cameras (constant) on a circle
    looking at vertical cylinders (tree trunks) around the origin; returns the
    scene (poses = ground truth) and the ground-truth cylinders [N][9]."""
    rng = np.random.default_rng(seed)
    f, cx, cy = 0.8 * width, width / 2.0, height / 2.0
    cams = np.tile([f, cx, cy], (num_images, 1))
    q = np.zeros((num_images, 4))
    t = np.zeros((num_images, 3))
    for i in range(num_images):
        a = 2 * np.pi * i / num_images + rng.uniform(-0.1, 0.1)
        centre = [9.0 * np.cos(a), 9.0 * np.sin(a), 1.5 + rng.uniform(-0.2, 0.2)]
        q[i], t[i] = look_at_qvec(centre, [rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), 2.0])
    cyl = np.zeros((num_cylinders, 9))
    for c in range(num_cylinders):
        a = 2 * np.pi * c / num_cylinders
        cyl[c, :4] = [1, 0, 0, 0]
        cyl[c, 4:7] = [2.2 * np.cos(a), 2.2 * np.sin(a), 0.0]
        cyl[c, 7] = rng.uniform(0.2, 0.4)
        cyl[c, 8] = rng.uniform(3.0, 4.5)
    X = rng.uniform(-3, 3, (points, 3)) + [0, 0, 2.0] if points else np.zeros((0, 3))
    xy, oi, op = [], [], []
    for p in range(points):
        for i in range(num_images):
            R = quat_to_rot(q[i])
            pc = R @ X[p] + t[i]
            if pc[2] <= 0.1:
                continue
            u, v = f * pc[0] / pc[2] + cx, f * pc[1] / pc[2] + cy
            if 0 <= u < width and 0 <= v < height:
                xy.append([u + rng.uniform(-1, 1), v + rng.uniform(-1, 1)])
                oi.append(i)
                op.append(p)
    sc = Scene(SIMPLE_PINHOLE, cams, q, t, np.arange(num_images, dtype=np.int32), np.asarray(X, float).reshape(-1, 3),
               np.asarray(xy, float).reshape(-1, 2), np.asarray(oi, np.int32), np.asarray(op, np.int32))
    sc.camera_constant = np.ones(num_images, np.uint8)
    return sc, cyl


def quat_to_rot(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


class Arena:
    """mi_ba_solve_in: consecutive solves on one recycled context."""

    def __init__(self):
        self.h = C.c_void_p(None)

    def solve(self, options: Options, scene: Scene, semantic: Optional[SemanticInput] = None) -> Summary:
        s = Summary()
        p = scene.problem()
        sem = semantic.struct() if semantic is not None else None
        check(load().mi_ba_solve_in(C.byref(self.h), C.cast(C.pointer(options), C.c_void_p),
                                    C.cast(C.pointer(p), C.c_void_p),
                                    None if sem is None else C.cast(C.pointer(sem), C.c_void_p),
                                    C.cast(C.pointer(s), C.c_void_p)), "mi_ba_solve_in")
        return s

    def close(self):
        if self.h.value:
            load().mi_ba_context_destroy(self.h)
            self.h = C.c_void_p(None)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def solve_batch(options, scenes, semantics=None, max_concurrent: int = 8):
    """mi_ba_solve_batch: independent problems solved concurrently; updates
    each scene in place.  options: one Options or one per scene.  Returns
    (statuses, summaries)."""
    n = len(scenes)
    opts = options if isinstance(options, (list, tuple)) else [options] * n
    O = (Options * n)(*opts)
    P = (Problem * n)(*[s.problem() for s in scenes])
    S = None
    keep = []
    if semantics is not None:
        structs = [None if x is None else x.struct() for x in semantics]
        keep = structs
        S = (C.c_void_p * n)(*[None if x is None else C.cast(C.pointer(x), C.c_void_p) for x in structs])
    sums = (Summary * n)()
    st = (C.c_int32 * n)()
    check(load().mi_ba_solve_batch(C.cast(O, C.c_void_p), C.cast(P, C.c_void_p), S and C.cast(S, C.c_void_p), n,
                                   max_concurrent, C.cast(sums, C.c_void_p), C.cast(st, C.c_void_p)),
          "mi_ba_solve_batch")
    del keep
    return list(st), list(sums)


def squared_reprojection_errors(scene: Scene, device: int = 0) -> np.ndarray:
    """CalculateSquaredReprojectionError of every observation (projection.cc:111-128)."""
    p = scene.problem()
    out = np.zeros(scene.num_obs)
    check(load().mi_ba_squared_reprojection_errors(C.byref(p), device, out.ctypes.data_as(_dp)),
          "mi_ba_squared_reprojection_errors")
    return out


def filter_points3d(scene: Scene, max_reproj_error: float, point_mask: Optional[np.ndarray] = None,
                    point_error: Optional[np.ndarray] = None, device: int = 0):
    """FilterPoints3DWithLargeReprojectionError (reconstruction.cc:1472-1525).
    Returns (obs_keep, point_keep, point_error, num_filtered)."""
    p = scene.problem()
    obs_keep = np.zeros(scene.num_obs, np.uint8)
    point_keep = np.zeros(scene.num_points, np.uint8)
    err = np.zeros(scene.num_points) if point_error is None else np.array(point_error, np.float64)
    mask = None if point_mask is None else np.ascontiguousarray(point_mask, dtype=np.uint8)
    nf = C.c_int64(0)
    check(load().mi_ba_filter_points3d(C.byref(p), max_reproj_error, _ptr(mask, _u8p), device,
                                       obs_keep.ctypes.data_as(_u8p), point_keep.ctypes.data_as(_u8p),
                                       err.ctypes.data_as(_dp), C.byref(nf)), "mi_ba_filter_points3d")
    return obs_keep.astype(bool), point_keep.astype(bool), err, nf.value


def positive_depth(scene: Scene, image_mask: Optional[np.ndarray] = None, device: int = 0):
    """mi_ba_positive_depth: (keep [N] bool, number of negative-depth
    observations) — FilterObservationsWithNegativeDepth's test."""
    p = scene.problem()
    keep = np.zeros(scene.num_obs, np.uint8)
    mask = None if image_mask is None else np.ascontiguousarray(image_mask, dtype=np.uint8)
    n = C.c_int64(0)
    check(load().mi_ba_positive_depth(C.byref(p), _ptr(mask, _u8p), device, keep.ctypes.data_as(_u8p), C.byref(n)),
          "mi_ba_positive_depth")
    return keep.astype(bool), n.value


def device_count() -> int:
    n = C.c_int32(0)
    load().mi_ba_device_count(C.byref(n))
    return n.value


def setup_stats(options: Options, scene: Scene) -> SetupInfo:
    info = SetupInfo()
    p = scene.problem()
    check(load().mi_ba_setup_stats(C.byref(options), C.byref(p), C.byref(info)), "mi_ba_setup_stats")
    return info


def solve(options: Options, scene: Scene, semantic: Optional[SemanticInput] = None) -> Summary:
    """BundleAdjuster::Solve on the device; updates scene arrays in place."""
    s = Summary()
    p = scene.problem()
    sem = semantic.struct() if semantic is not None else None
    st = load().mi_ba_solve(C.byref(options), C.byref(p), C.byref(sem) if sem is not None else None, C.byref(s))
    check(st, "mi_ba_solve")
    return s


class Context:
    """Device-resident problem (mi_ba_context_*)."""

    def __init__(self, options: Options, scene: Scene, semantic: Optional[SemanticInput] = None):
        self.lib = load()
        self.options = options
        self.scene = scene
        self.semantic = semantic
        self._p = scene.problem()
        self._s = semantic.struct() if semantic is not None else None
        h = C.c_void_p()
        check(self.lib.mi_ba_context_create(C.byref(options), C.byref(self._p),
                                            C.byref(self._s) if self._s is not None else None, C.byref(h)),
              "mi_ba_context_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.mi_ba_context_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def dims(self):
        nb, cols, ns = C.c_int64(), C.c_int32(), C.c_int64()
        check(self.lib.mi_ba_context_dims(self.h, C.byref(nb), C.byref(cols), C.byref(ns)), "dims")
        return nb.value, cols.value, ns.value

    def linearize(self):
        check(self.lib.mi_ba_linearize(self.h), "mi_ba_linearize")

    def evaluate_jacobian(self):
        check(self.lib.mi_ba_evaluate_jacobian(self.h), "mi_ba_evaluate_jacobian")

    def evaluate_semantic(self):
        check(self.lib.mi_ba_evaluate_semantic(self.h), "mi_ba_evaluate_semantic")

    def synchronize(self):
        check(self.lib.mi_ba_synchronize(self.h), "mi_ba_synchronize")

    def download_jacobian(self):
        nb, cols, _ = self.dims()
        bo = np.empty(nb, np.int64)
        r = np.empty((nb, 2), np.float64)
        J = np.empty((nb, 2, cols), np.float64)
        check(self.lib.mi_ba_download_jacobian(self.h, _ptr(bo, _i64p), _ptr(r, _dp), _ptr(J, _dp)), "download")
        return bo, r, J

    def download_semantic(self):
        _, _, ns = self.dims()
        px = np.empty((ns, 3), np.int32)
        st = np.empty(ns, np.int32)
        r = np.empty(ns, np.float64)
        J = np.empty((ns, 12), np.float64)
        check(self.lib.mi_ba_download_semantic(self.h, _ptr(px, _i32p), _ptr(st, _i32p), _ptr(r, _dp),
                                               _ptr(J, _dp)), "download_semantic")
        return px, st, r, J

    def semantic_export(self, image1: int, image2: int):
        """mi_ba_semantic_export: ExportSemanticErrorToCSV's rows of the ordered
        image pair at the current parameters -> (pixels [n][4] (x1, y1, x2, y2),
        status [n], error [n], world [n][3])."""
        n = C.c_int64(0)
        check(self.lib.mi_ba_semantic_export(self.h, image1, image2, C.byref(n), None, None, None, None),
              "mi_ba_semantic_export")
        pix = np.empty((n.value, 4), np.int32)
        st = np.empty(n.value, np.int32)
        err = np.empty(n.value, np.float64)
        world = np.empty((n.value, 3), np.float64)
        check(self.lib.mi_ba_semantic_export(self.h, image1, image2, C.byref(n), _ptr(pix, _i32p), _ptr(st, _i32p),
                                             _ptr(err, _dp), _ptr(world, _dp)), "mi_ba_semantic_export")
        return pix, st, err, world

    def solve(self) -> Summary:
        s = Summary()
        check(self.lib.mi_ba_context_solve(self.h, C.byref(s)), "mi_ba_context_solve")
        return s

    def writeback(self):
        check(self.lib.mi_ba_context_writeback(self.h), "mi_ba_context_writeback")

    def cost(self) -> float:
        c = C.c_double()
        check(self.lib.mi_ba_context_cost(self.h, C.byref(c)), "cost")
        return c.value

    def set_tuning(self, key: str, value: int):
        check(self.lib.mi_ba_set_tuning(self.h, key.encode(), int(value)), "set_tuning")

    def set_timing(self, on: bool):
        check(self.lib.mi_ba_set_timing(self.h, 1 if on else 0), "timing")

    def kernel_time(self, name: str):
        ms, n = C.c_double(), C.c_int64()
        check(self.lib.mi_ba_kernel_time(self.h, name.encode(), C.byref(ms), C.byref(n)), "kernel_time")
        return ms.value, n.value

    def reset_kernel_times(self):
        check(self.lib.mi_ba_reset_kernel_times(self.h), "reset")

    # multi-rank LM ------------------------------------------------------
    def set_comm(self, rank: int, world: int, unique_id: bytes):
        """Join an RCCL communicator (one process per GPU)."""
        check(self.lib.mi_ba_context_set_comm(self.h, rank, world, bytes(unique_id).ljust(COMM_ID_BYTES, b"\0")),
              "mi_ba_context_set_comm")

    def set_host_reducer(self, rank: int, world: int, reduce_inplace):
        """Join a multi-rank solve whose sums go through `reduce_inplace(np.ndarray)`
        (e.g. a torch.distributed gloo all-reduce); for ranks sharing a GPU."""
        def _cb(ptr, n, _user):
            try:
                reduce_inplace(np.ctypeslib.as_array(ptr, shape=(n,)))
                return 0
            except Exception:  # noqa: BLE001 — reported to the library as a failed reduction
                return 1
        self._reducer = HOST_ALLREDUCE_FN(_cb)  # keep the thunk alive
        check(self.lib.mi_ba_context_set_host_reducer(self.h, rank, world, self._reducer, None),
              "mi_ba_context_set_host_reducer")


# ---------------------------------------------------------------------------
# synthetic scenes (include/mi_ba_synthetic.h)
# ---------------------------------------------------------------------------
def synth_config(camera_model=SIMPLE_RADIAL, num_images=2, num_points=100, track_length=0, image_size=1000,
                 focal_factor=1.2, extra=(0.0, 0.0, 0.0, 0.0), rotation_range=0.0, noise=2.0, seed=0):
    c = SynthConfig()
    c.camera_model = camera_model
    c.num_images = num_images
    c.num_points = num_points
    c.track_length = track_length
    c.image_size = image_size
    c.focal_factor = focal_factor
    for k in range(4):
        c.extra[k] = extra[k] if k < len(extra) else 0.0
    c.rotation_range = rotation_range
    c.noise = noise
    c.seed = seed
    return c


def convert_cameras(scene: Scene, models) -> Scene:
    """Give camera c the model models[c % len(models)] (a mixed-model
    reconstruction): the SIMPLE_RADIAL parameters (f, cx, cy, k) of a
    generated scene are carried over to the other models' layouts
    (camera_models.h *Idxs), with small second-order distortion terms."""
    assert scene.camera_model == SIMPLE_RADIAL and scene.camera_models is None
    ids, params = [], []
    for c in range(scene.num_cameras):
        f, cx, cy, k = scene.camera_params[c]
        m = int(models[c % len(models)])
        ids.append(m)
        params.extend({SIMPLE_PINHOLE: [f, cx, cy], PINHOLE: [f, f * 1.01, cx, cy], SIMPLE_RADIAL: [f, cx, cy, k],
                       RADIAL: [f, cx, cy, k, -0.01], OPENCV: [f, f * 0.99, cx, cy, k, 0.01, 1e-4, -1e-4]}[m])
    out = scene.copy()
    out.camera_models = np.array(ids, np.int32)
    out.camera_params = np.array(params, np.float64)
    return out


def generate_scene(cfg: SynthConfig) -> Scene:
    lib = load_synth()
    n = lib.mi_ba_synth_num_obs(C.byref(cfg))
    I, P = cfg.num_images, cfg.num_points
    npar = NUM_PARAMS[cfg.camera_model]
    cam = np.zeros((I, npar))
    q = np.zeros((I, 4))
    t = np.zeros((I, 3))
    ic = np.zeros(I, np.int32)
    X = np.zeros((P, 3))
    xy = np.zeros((n, 2))
    oi = np.zeros(n, np.int32)
    op = np.zeros(n, np.int32)
    st = lib.mi_ba_synth_generate(C.byref(cfg), _ptr(cam, _dp), _ptr(q, _dp), _ptr(t, _dp), _ptr(ic, _i32p),
                                  _ptr(X, _dp), _ptr(xy, _dp), _ptr(oi, _i32p), _ptr(op, _i32p))
    if st != 0:
        raise RuntimeError("mi_ba_synth_generate failed")
    return Scene(cfg.camera_model, cam, q, t, ic, X, xy, oi, op)


def render_semantic(scene: Scene, height: int, width: int, plane_z: float = 1.0, cell: float = 0.1):
    lib = load_synth()
    I = scene.num_images
    scene._normalize()
    depth = np.zeros((I, height, width), np.float32)
    label = np.zeros((I, height, width), np.float32)
    if scene.camera_models is not None:  # mixed models: one image at a time with its camera's model
        off = scene.camera_param_offsets()
        for i in range(I):
            c = int(scene.image_camera[i])
            one = Scene(int(scene.camera_models[c]), scene.camera_params[off[c]:off[c + 1]][None, :].copy(),
                        scene.qvec[i:i + 1].copy(), scene.tvec[i:i + 1].copy(), np.zeros(1, np.int32),
                        scene.xyz[:0], scene.obs_xy[:0], scene.obs_image[:0], scene.obs_point[:0])
            d, l_ = render_semantic(one, height, width, plane_z, cell)
            depth[i], label[i] = d[0], l_[0]
        return depth, label
    st = lib.mi_ba_synth_render(scene.camera_model, I, _ptr(scene.camera_params, _dp), _ptr(scene.qvec, _dp),
                                _ptr(scene.tvec, _dp), _ptr(scene.image_camera, _i32p), height, width, plane_z,
                                cell, _ptr(depth, _fp), _ptr(label, _fp))
    if st != 0:
        raise RuntimeError("mi_ba_synth_render failed")
    return depth, label
