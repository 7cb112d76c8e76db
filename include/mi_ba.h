/*
 * mi_ba.h — C-ABI drop-in boundary of the MI355X-native semantic bundle
 * adjustment hot path.
 *
 * Every entry point here replaces one piece of the reference's C++ interface
 * (AlainSchoebi/semantic-bundle-adjustment-colmap, a COLMAP 3.8 fork):
 *
 *   mi_ba_default_options      <- BundleAdjustmentOptions::BundleAdjustmentOptions()
 *                                 src/optim/bundle_adjustment.h:49-92
 *   mi_ba_problem (struct)     <- Reconstruction (cameras/images/points3D/tracks)
 *                                 + BundleAdjustmentConfig (bundle_adjustment.h:103-167)
 *                                 flattened the way ParallelBundleAdjuster::SetUp does
 *                                 (src/optim/bundle_adjustment.cc:665-783)
 *   mi_ba_setup_stats          <- BundleAdjuster::SetUp + Ceres reduced-program counts
 *                                 (bundle_adjustment.cc:326-530; summary fields read by
 *                                 src/optim/bundle_adjustment_test.cc:186-642)
 *   mi_ba_solve                <- BundleAdjuster::Solve(Reconstruction*) + Summary()
 *                                 (bundle_adjustment.h:171-203, bundle_adjustment.cc:258-320)
 *   mi_ba_context_* / mi_ba_linearize / mi_ba_download_*
 *                              <- the Ceres residual+Jacobian evaluation of every
 *                                 BundleAdjustmentCostFunction /
 *                                 BundleAdjustmentConstantPoseCostFunction block
 *                                 (src/base/cost_functions.h:44-152) and of every
 *                                 {,ConstantFirstPose,ConstantSecondPose}SemanticBACostFunction
 *                                 block (src/base/semantic_cost_functions.h:87-404),
 *                                 reduced into Schur normal equations (Ceres 2.1
 *                                 SchurEliminator, 3rd party, not vendored)
 *   mi_ba_squared_reprojection_errors / mi_ba_filter_points3d
 *                              <- CalculateSquaredReprojectionError (src/base/projection.cc:111-128),
 *                                 Reconstruction::FilterPoints3DWithLargeReprojectionError
 *                                 (src/base/reconstruction.cc:1472-1525)
 *   mi_ba_semantic (struct)    <- SemanticBundleAdjustmentOptions depth/semantic maps
 *                                 (src/optim/semantic_bundle_adjustment.h:53-140,
 *                                 semantic_bundle_adjustment.cc:699-906,1021-1068)
 *
 * Conventions: caller owns every host array; arrays marked (in/out) are
 * updated in place by mi_ba_solve exactly where Ceres would mutate the
 * Reconstruction through its registered double* parameter blocks
 * (bundle_adjustment.cc:357-359,393,408-410).  Errors are returned as
 * mi_ba_status codes (the reference aborts through glog CHECK or throws).
 * Device buffers are library-owned.  One context per host thread.
 * All arithmetic is IEEE f64.
 */
#ifndef MI_BA_H_
#define MI_BA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI_BA_ABI_VERSION 4

typedef enum mi_ba_status {
  MI_BA_OK = 0,
  MI_BA_ERR_INVALID_ARGUMENT = 1, /* reference: glog CHECK abort (bundle_adjustment.cc:165-186,304) */
  MI_BA_ERR_NO_DEVICE = 2,        /* no MI355X visible: the product never falls back to the CPU */
  MI_BA_ERR_UNSUPPORTED = 3,      /* reference: std::domain_error / std::runtime_error */
  MI_BA_ERR_HIP = 4,              /* HIP runtime error */
  MI_BA_ERR_NO_RESIDUALS = 5,     /* reference: Solve() returns false (bundle_adjustment.cc:267-269) */
  MI_BA_ERR_STATE = 6,            /* reference: "Cannot use the same BundleAdjuster multiple times" */
  MI_BA_ERR_OUT_OF_MEMORY = 7
} mi_ba_status;

/* COLMAP camera model ids (src/base/camera_models.h kModelId). */
enum {
  MI_BA_SIMPLE_PINHOLE = 0,
  MI_BA_PINHOLE = 1,
  MI_BA_SIMPLE_RADIAL = 2,
  MI_BA_RADIAL = 3,
  MI_BA_OPENCV = 4
};

/* BundleAdjustmentOptions::LossFunctionType (bundle_adjustment.h:51). */
enum { MI_BA_LOSS_TRIVIAL = 0, MI_BA_LOSS_SOFT_L1 = 1, MI_BA_LOSS_CAUCHY = 2 };

/* Linear solver selection; AUTO reproduces the heuristic of
 * bundle_adjustment.cc:276-286 (<=50 images dense Schur, else iterative). */
enum {
  MI_BA_SOLVER_AUTO = 0,
  MI_BA_SOLVER_DENSE_SCHUR = 1,
  MI_BA_SOLVER_ITERATIVE_SCHUR = 2
};

/* ceres::TerminationType, same numeric order as Ceres 2.1. */
enum {
  MI_BA_CONVERGENCE = 0,
  MI_BA_NO_CONVERGENCE = 1,
  MI_BA_FAILURE = 2,
  MI_BA_USER_SUCCESS = 3,
  MI_BA_USER_FAILURE = 4
};

/* ceres::CallbackReturnType, same numeric order as Ceres 2.1: what an
 * iteration callback (or the stop flag) asks of the solver. */
enum {
  MI_BA_SOLVER_CONTINUE = 0,
  MI_BA_SOLVER_ABORT = 1,                  /* -> termination_type MI_BA_USER_FAILURE; the
                                              problem arrays are not updated (Ceres) */
  MI_BA_SOLVER_TERMINATE_SUCCESSFULLY = 2  /* -> termination_type MI_BA_USER_SUCCESS */
};

/* ceres::IterationSummary fields, handed to the iteration callback at the end
 * of every LM iteration (TrustRegionMinimizer::
 * FinalizeIterationAndCheckIfMinimizerCanContinue): iteration 0 is the
 * initial state (after the first residual + Jacobian evaluation), then one
 * per iteration, successful, unsuccessful or invalid.  Iterations that end
 * the solve on a tolerance or on too many invalid steps run no callback
 * (Ceres returns from those before the callbacks). */
typedef struct mi_ba_iteration_summary {
  int32_t iteration;
  int32_t step_is_valid;
  int32_t step_is_successful;
  int32_t linear_solver_iterations;
  double cost;                        /* at the current (accepted) point, fixed cost included */
  double cost_change;                 /* cost - candidate cost of every valid step (negative when
                                         rejected, as Ceres); 0 for an invalid step */
  double relative_decrease;
  double trust_region_radius;         /* after this iteration's update */
  double step_norm;
  double iteration_time_in_seconds;
  double cumulative_time_in_seconds;
} mi_ba_iteration_summary;

/* ceres::IterationCallback::operator(): returns MI_BA_SOLVER_*.  Runs on the
 * thread that called the solve.  With options.update_state_every_iteration
 * the problem's parameter arrays (qvec, tvec, xyz, camera_params, cylinders)
 * hold the current point when it runs (Ceres' update_state_every_iteration,
 * which the reference's SBA / GSBA snapshot callbacks rely on,
 * semantic_bundle_adjustment.h:129, semantic_bundle_adjustment.cc:1086-1123). */
typedef int32_t (*mi_ba_iteration_callback_fn)(void* user, const mi_ba_iteration_summary* summary);

/* Semantic sample status (ReprojectionStatus, semantic_cost_functions.h:45). */
enum { MI_BA_OUT_OF_BOUNDS = -1, MI_BA_INVALID_DEPTH = -2, MI_BA_VALID = 10 };

typedef struct mi_ba_options {
  int32_t loss_function_type;       /* MI_BA_LOSS_*; default TRIVIAL */
  double loss_function_scale;       /* default 1.0 */
  int32_t refine_focal_length;      /* default 1 */
  int32_t refine_principal_point;   /* default 0 */
  int32_t refine_extra_params;      /* default 1 */
  int32_t refine_extrinsics;        /* default 1 */
  int32_t print_summary;            /* default 0 (library does not print unless asked) */
  /* ceres::Solver::Options subset set by BundleAdjustmentOptions() */
  int32_t max_num_iterations;       /* 100 */
  double function_tolerance;        /* 0 */
  double gradient_tolerance;        /* 0 */
  double parameter_tolerance;       /* 0 */
  int32_t max_linear_solver_iterations;      /* 200 */
  int32_t max_num_consecutive_invalid_steps; /* 10 */
  int32_t linear_solver_type;       /* MI_BA_SOLVER_AUTO */
  double eta;                       /* inexact-Newton forcing, Ceres default 0.1 */
  double initial_trust_region_radius; /* Ceres default 1e4 */
  double min_relative_decrease;     /* Ceres default 1e-3 */
  /* build additions */
  int32_t device;                   /* HIP device ordinal, default 0 */
  double semantic_weight;           /* ScaledLoss weight of semantic blocks, default 1 */
  /* solver_options.callbacks / update_state_every_iteration (ABI 3): the
   * reference's controllers install an IterationCallback that blocks while
   * the thread is paused and returns SOLVER_TERMINATE_SUCCESSFULLY once it is
   * stopped (controllers/bundle_adjustment.cc:43-61,87-88). */
  mi_ba_iteration_callback_fn iteration_callback; /* nullable, default NULL */
  void* callback_user;
  int32_t update_state_every_iteration;           /* default 0 */
  /* Stop flag, nullable: read (atomically, relaxed) where the callback runs;
   * a nonzero value is taken as that callback return (MI_BA_SOLVER_*), so
   * another thread stops the solve at the next iteration boundary by
   * storing MI_BA_SOLVER_TERMINATE_SUCCESSFULLY (Thread::Stop) or
   * MI_BA_SOLVER_ABORT. */
  const int32_t* stop_flag;
} mi_ba_options;

/* Flattened Reconstruction + BundleAdjustmentConfig.  Indices are 0-based
 * positions in these arrays.  Camera models: camera_model_ids[c] per camera
 * (Camera::ModelId, dispatched per camera like camera_models.h:117-141), or,
 * when camera_model_ids is NULL, camera_model for every camera.
 * camera_params holds each camera's Camera::Params() back to back in camera
 * order (num_params(model of camera c) doubles each; with one model this is
 * [num_cameras][num_params(model)]). */
typedef struct mi_ba_problem {
  int32_t camera_model;              /* MI_BA_* model id of every camera when camera_model_ids is NULL */
  int32_t num_cameras;
  double* camera_params;             /* (in/out) per-camera params, back to back */
  const uint8_t* camera_constant;    /* nullable; 1 = config.SetConstantCamera */

  int32_t num_images;
  double* qvec;                      /* (in/out) [num_images][4] (w,x,y,z), world->camera */
  double* tvec;                      /* (in/out) [num_images][3] */
  const int32_t* image_camera;       /* [num_images] camera index */
  const uint8_t* image_in_config;    /* nullable (= all); 1 = config.AddImage */
  const uint8_t* image_constant_pose;/* nullable; 1 = config.SetConstantPose */
  const uint8_t* image_constant_tvec;/* nullable; bit k = tvec[k] constant (config.SetConstantTvec) */

  int64_t num_points;
  double* xyz;                       /* (in/out) [num_points][3] */
  const uint8_t* point_config;       /* nullable; 1 = AddVariablePoint, 2 = AddConstantPoint */

  int64_t num_obs;                   /* all track elements of the reconstruction */
  const double* obs_xy;              /* [num_obs][2] Point2D::XY() */
  const int32_t* obs_image;          /* [num_obs] */
  const int32_t* obs_point;          /* [num_obs] */
  const int32_t* camera_model_ids;   /* nullable; [num_cameras] MI_BA_* model id per camera (ABI 2) */
} mi_ba_problem;

/* Semantic term (SBA).  Rasters are row-major float32, i.e. the
 * Eigen::MatrixXf (row=y, col=x) of matrixFromTiff after its vertical flip
 * (matrix_vis.h:130-176).  An image's depth and semantic maps share one size.
 * Sizes (ABI 4): with image_height / image_width NULL every image is
 * height x width and depth / label are [num_images][height][width]; else
 * image i is image_height[i] x image_width[i] (height / width are ignored)
 * and depth / label hold the images' planes back to back in image order
 * (plane i starts at sum_{k<i} H_k W_k).  As the reference
 * (semantic_bundle_adjustment.cc:792-799, semantic_cost_functions.h:163),
 * image i of a pair is sampled on its own H_i x W_i grid and the reprojected
 * pixel is bounds-checked against image j's own H_j x W_j.  Every image of a
 * pair needs H, W > 0 (MI_BA_ERR_INVALID_ARGUMENT otherwise). */
typedef struct mi_ba_semantic {
  int32_t height;
  int32_t width;
  const float* depth;                /* image planes, see above */
  const float* label;                /* image planes, see above */
  int32_t num_pairs;                 /* ordered pairs (i, j); reference uses all i != j */
  const int32_t* pairs;              /* [num_pairs][2] */
  int32_t pixel_step;                /* error_computation_pixel_step, default 10 */
  double depth_error_threshold;      /* default 2 */
  double numeric_relative_step_size; /* default 1e-3 */
  const int32_t* image_height;       /* nullable [num_images] (ABI 4) */
  const int32_t* image_width;        /* nullable [num_images] (ABI 4) */
} mi_ba_semantic;

/* Geometric-semantic BA (GSBA): one cylinder IoU residual per (config image,
 * cylinder) (GeometricSemanticBundleAdjuster<Cylinder>,
 * src/optim/geometric_semantic_bundle_adjustment.{h,cc}; residual 1 - IoU of
 * the cylinder's projected quadrilateral against the image's trunk mask,
 * Cylinder::ComputeSemanticIoU src/util/cylinder.h:496-540; CENTRAL numeric
 * derivatives, geometric_semantic_cost_functions.h:33-165), ScaledLoss(1 /
 * number of config images).  Requirements as GeometricSemanticBundleAdjuster::
 * Assert (:664-712): config cameras constant and SIMPLE_PINHOLE, TRIVIAL loss
 * (else MI_BA_ERR_UNSUPPORTED).  Cylinders: QuaternionManifold on qvec,
 * radius bounded below by 0 (the reference sets the "height" bound on the
 * radius block, :1180). */
typedef struct mi_ba_cylinder {
  double qvec[4];                    /* (w,x,y,z) cylinder -> world rotation (Cylinder::Qvec) */
  double tvec[3];                    /* lower circle centre in the world */
  double radius;
  double height;
} mi_ba_cylinder;

/* GeometricSemanticBundleAdjustmentOptions::cylinder_parametrization
 * (geometric_semantic_bundle_adjustment.h:49-95): "default" optimises each
 * cylinder as (qvec 4 on the QuaternionManifold, tvec 3, radius, height);
 * "by_2_points" as CylinderBy2Points (src/util/cylinder_by_2_points.h:26-155):
 * the centres of its two circles and its radius, Euclidean, radius bounded
 * below by 0 (:1185-1213), evaluated through CylinderBy2Points::ToCylinder.
 * The cylinders are read and written as (qvec, tvec, radius, height) in both
 * (pushBackCylindersReadFromText / exportCylindersToText). */
enum { MI_BA_CYLINDER_DEFAULT = 0, MI_BA_CYLINDER_BY_2_POINTS = 1 };

typedef struct mi_ba_gsba {
  int32_t height;                    /* trunk mask size of every image (image_height NULL) */
  int32_t width;
  const uint8_t* trunk_mask;         /* row-major, 1 where the semantic map == trunk_semantic_class
                                        (:1328-1333), images in problem order: [num_images][H][W], or
                                        with image_height / image_width the planes back to back */
  int32_t num_cylinders;
  mi_ba_cylinder* cylinders;         /* (in/out) */
  int32_t refine_geometry;           /* default 1 */
  double numeric_relative_step_size; /* default 1e-3 */
  int32_t include_landmark_error;    /* default 0: the problem's observations are not used */
  double landmark_error_weight;      /* default 1: reprojection blocks get ScaledLoss(w / #config 2D features) */
  int32_t cylinder_parametrization;  /* MI_BA_CYLINDER_*, default MI_BA_CYLINDER_DEFAULT (ABI 3) */
  /* nullable [num_images] per-image mask sizes (ABI 4): each image's IoU is
   * rasterised on its own semantic map's size (Cylinder::ComputeSemanticIoU
   * takes the map's rows / cols, cylinder.h:496-504;
   * geometric_semantic_bundle_adjustment.cc:1530-1531) */
  const int32_t* image_height;
  const int32_t* image_width;
} mi_ba_gsba;

/* Mirrors the ceres::Solver::Summary fields COLMAP reads
 * (PrintSolverSummary, bundle_adjustment.cc:1142-1196). */
typedef struct mi_ba_summary {
  int64_t num_residuals_reduced;
  int64_t num_effective_parameters_reduced;
  int32_t num_successful_steps;
  int32_t num_unsuccessful_steps;
  int32_t termination_type;
  double initial_cost;
  double final_cost;
  double fixed_cost;
  double total_time_in_seconds;
  double jacobian_evaluation_time_in_seconds;
  int32_t num_jacobian_evaluations;
  int32_t num_linear_solver_iterations;
  int64_t num_semantic_residuals;
} mi_ba_summary;

/* Structural counts produced by problem assembly (no device needed). */
typedef struct mi_ba_setup_info {
  int64_t num_residual_blocks;          /* geometric blocks in the program */
  int64_t num_residuals_reduced;        /* after dropping all-constant blocks */
  int64_t num_effective_parameters_reduced;
  int64_t num_variable_images;
  int64_t num_variable_cameras;
  int64_t num_variable_points;
  int32_t camera_tangent_size;          /* refined intrinsics per camera */
} mi_ba_setup_info;

typedef struct mi_ba_context mi_ba_context;

/* --- version / device --------------------------------------------------- */
int32_t mi_ba_abi_version(void);
const char* mi_ba_status_string(int32_t status);
int32_t mi_ba_num_params(int32_t camera_model); /* -1 if unknown */
mi_ba_status mi_ba_device_count(int32_t* count);

/* --- options ------------------------------------------------------------ */
void mi_ba_default_options(mi_ba_options* options);

/* --- problem assembly (host only) -------------------------------------- */
mi_ba_status mi_ba_setup_stats(const mi_ba_options* options,
                               const mi_ba_problem* problem,
                               mi_ba_setup_info* info);

/* --- one-shot solve: BundleAdjuster::Solve ------------------------------
 * The refined parameters are written into the problem arrays unless the
 * solve ends in MI_BA_FAILURE or MI_BA_USER_FAILURE, where Ceres leaves the
 * user's parameter blocks untouched (Solver::Solve copies the state back only
 * for a usable solution); with update_state_every_iteration they then hold
 * the point of the last callback. */
mi_ba_status mi_ba_solve(const mi_ba_options* options, mi_ba_problem* problem,
                         const mi_ba_semantic* semantic /* nullable */,
                         mi_ba_summary* summary);

/* --- geometric-semantic BA (GSBA) ----------------------------------------
 * mi_ba_default_gsba: GeometricSemanticBundleAdjustmentOptions defaults.
 * mi_ba_gsba_solve: GeometricSemanticBundleAdjuster<Cylinder> (or
 * <CylinderBy2Points>, gsba.cylinder_parametrization)::Solve on the
 * GPU: poses (and cylinders when refine_geometry) refined; with
 * include_landmark_error also the problem's points (SIMPLE_PINHOLE
 * reprojection blocks, ScaledLoss).  Blocks are ordered by config image
 * (problem order) then cylinder.
 * mi_ba_gsba_evaluate: residual 1 - IoU and the ambient CENTRAL Jacobian
 * [n][16] (camera q(4) t(3), cylinder q(4) t(3) radius height — by_2_points:
 * cylinder tvec_1(3) tvec_2(3) radius and two zero columns; columns of
 * constant blocks zero) of every block, before the ScaledLoss; block_ids
 * [n][2] = (image, cylinder).  *num_blocks receives the count; nothing is
 * written when it exceeds capacity. */
void mi_ba_default_gsba(mi_ba_gsba* gsba);
mi_ba_status mi_ba_gsba_solve(const mi_ba_options* options, mi_ba_problem* problem, mi_ba_gsba* gsba,
                              mi_ba_summary* summary);
mi_ba_status mi_ba_gsba_evaluate(const mi_ba_options* options, mi_ba_problem* problem, const mi_ba_gsba* gsba,
                                 int64_t capacity, int64_t* num_blocks, int32_t* block_ids,
                                 double* residuals, double* jacobians);

/* --- repeated solves (the incremental mapper's local / global BAs) -------
 * As mi_ba_solve, on the context in *arena (NULL: one is created) whose
 * device resources — stream, rocBLAS handles, Cholesky workspace, device
 * arrays large enough for the new problem — are reused; the context stays
 * in *arena for the next call (NULL after a failed call).  Release it with
 * mi_ba_context_destroy.  One arena per host thread. */
mi_ba_status mi_ba_solve_in(mi_ba_context** arena, const mi_ba_options* options, mi_ba_problem* problem,
                            const mi_ba_semantic* semantic /* nullable */, mi_ba_summary* summary);

/* --- many independent problems (incremental-mapper local BAs, submodels) -
 * Solves problems[k] with options[k] (and semantics[k] when semantics is not
 * NULL) for k < n, as mi_ba_solve would one after the other, with up to
 * max_concurrent (<= 0: 8) solves in flight on their own contexts and HIP
 * streams.  statuses[k] / summaries[k] are mi_ba_solve's per problem; the
 * call itself fails only on invalid arguments.  Problems must not share
 * arrays they write (parameters). */
mi_ba_status mi_ba_solve_batch(const mi_ba_options* options, mi_ba_problem* problems,
                               const mi_ba_semantic* const* semantics /* nullable */, int32_t n,
                               int32_t max_concurrent, mi_ba_summary* summaries, int32_t* statuses);

/* --- reprojection errors and track filtering (host buffers in and out) --
 * mi_ba_squared_reprojection_errors: CalculateSquaredReprojectionError
 * (src/base/projection.cc:111-128) of every observation at the problem's
 * current parameters; DBL_MAX where the point is behind the camera
 * (z < DBL_EPSILON).  qvec need not be normalised (QuaternionRotatePoint
 * normalises).
 * mi_ba_filter_points3d: Reconstruction::FilterPoints3DWithLargeReprojectionError
 * (src/base/reconstruction.cc:1472-1525) over the points with point_mask[p]
 * != 0 (NULL = every point): a point's observations with squared error above
 * max_reproj_error^2 are dropped (obs_keep[k] = 0); a point left with fewer
 * than two (or with a track shorter than two) is deleted (point_keep[p] = 0,
 * all its observations dropped); otherwise point_error[p] = mean
 * reprojection error of the kept observations (unmasked and deleted points
 * keep the caller's value).  *num_filtered = observations dropped, as the
 * reference's return value.  A point's observations are visited in problem
 * order (the flatteners emit them in Track order). */
mi_ba_status mi_ba_squared_reprojection_errors(const mi_ba_problem* problem, int32_t device,
                                               double* sq_errors);
mi_ba_status mi_ba_filter_points3d(const mi_ba_problem* problem, double max_reproj_error,
                                   const uint8_t* point_mask /* nullable */, int32_t device,
                                   uint8_t* obs_keep, uint8_t* point_keep, double* point_error,
                                   int64_t* num_filtered);

/* mi_ba_positive_depth: the test of Reconstruction::
 * FilterObservationsWithNegativeDepth (src/base/reconstruction.cc:647-665),
 * the pre-step every BA controller runs before Solve
 * (controllers/bundle_adjustment.cc:82, semantic_bundle_adjustment.cc:86,
 * geometric_semantic_bundle_adjustment.cc:89): obs_keep[k] = 1 when
 * HasPointPositiveDepth(ProjectionMatrix of the observation's image, its
 * point) (projection.cc:191-195: third row of [R(normalised qvec) | t] dotted
 * with (X, 1) >= DBL_EPSILON), 0 otherwise; observations of images with
 * image_mask[i] == 0 (NULL = every image; the reference visits the registered
 * images) are kept.  *num_negative = observations with obs_keep 0.  The
 * reference then deletes those observations one by one in image / point2D
 * order, a track of length <= 2 taking its point with it
 * (Reconstruction::DeleteObservation, reconstruction.cc:257-277); the facade
 * (colmap_amd::Reconstruction::FilterObservationsWithNegativeDepth) applies
 * the mask that way. */
mi_ba_status mi_ba_positive_depth(const mi_ba_problem* problem, const uint8_t* image_mask /* nullable */,
                                  int32_t device, uint8_t* obs_keep, int64_t* num_negative);

/* --- resident context (device-resident problem, for throughput/parity) - */
mi_ba_status mi_ba_context_create(const mi_ba_options* options,
                                  const mi_ba_problem* problem,
                                  const mi_ba_semantic* semantic /* nullable */,
                                  mi_ba_context** ctx);
void mi_ba_context_destroy(mi_ba_context* ctx);

/* Residual + Jacobian evaluation of every block at the current parameters,
 * reduced into the Schur normal-equation blocks.  Asynchronous on the
 * context's stream; call mi_ba_synchronize before reading results. */
mi_ba_status mi_ba_linearize(mi_ba_context* ctx);
/* Residual+Jacobian kernel alone (the J-materialising evaluation). */
mi_ba_status mi_ba_evaluate_jacobian(mi_ba_context* ctx);
/* Semantic residual+Jacobian kernel alone, also storing the per-sample
 * residual / status / Jacobian for mi_ba_download_semantic (the solver's
 * linearization reduces them into pair blocks without storing them). */
mi_ba_status mi_ba_evaluate_semantic(mi_ba_context* ctx);
mi_ba_status mi_ba_synchronize(mi_ba_context* ctx);

/* Number of geometric residual blocks in the context (rows of the download
 * arrays below) and the per-block Jacobian width 9 + camera_tangent_size. */
mi_ba_status mi_ba_context_dims(const mi_ba_context* ctx, int64_t* num_blocks,
                                int32_t* jacobian_cols, int64_t* num_samples);
/* Blocks are in the library's point-major order; block_obs[k] = index of
 * the problem observation evaluated by block k.  Layout:
 *   residuals [num_blocks][2]
 *   jacobian  [num_blocks][2][9+c] columns: rot(3 tangent) trans(3) point(3)
 *             cam(c refined intrinsics); columns of constant parameter blocks
 *             and constant tvec coordinates are zero. */
mi_ba_status mi_ba_download_jacobian(mi_ba_context* ctx, int64_t* block_obs,
                                     double* residuals, double* jacobian);
/* Semantic samples of the last mi_ba_evaluate_semantic (MI_BA_ERR_STATE
 * when the last semantic evaluation did not store them), ordered by pair then (y, x):
 *   sample_pixel [n][3] (pair index, x1, y1); status [n]; residual [n];
 *   jacobian [n][12] = pose1 (rot3, trans3), pose2 (rot3, trans3). */
mi_ba_status mi_ba_download_semantic(mi_ba_context* ctx, int32_t* sample_pixel,
                                     int32_t* status, double* residuals,
                                     double* jacobian);
/* The rows of SemanticBundleAdjuster::ExportSemanticErrorToCSV
 * (semantic_bundle_adjustment.cc:908-1019) for the ordered image pair
 * (image1, image2) — problem image indices — at the context's current
 * parameters (inside an iteration callback: the current LM point): every
 * pixel of image1's grid, y outer / x inner with the semantic pixel_step,
 * zero-depth pixels included (the reference exports them; the problem's
 * samples skip them), through compute_semantic_error
 * (semantic_cost_functions.h:87-208).  *count = number of grid pixels;
 * with pixels == NULL only the count is returned.  Rows:
 *   pixels [n][4] (X1, Y1, X2, Y2: image1 pixel, rounded image2 pixel);
 *   status [n] (MI_BA_VALID / _OUT_OF_BOUNDS / _INVALID_DEPTH);
 *   error [n] (0 / 1); world [n][3] (the image1 pixel's point in world).
 * MI_BA_ERR_UNSUPPORTED when either image's rasters are not resident (an
 * image that is the second image of no configured pair). */
mi_ba_status mi_ba_semantic_export(mi_ba_context* ctx, int32_t image1, int32_t image2, int64_t* count,
                                   int32_t* pixels, int32_t* status, double* error, double* world);
/* LM solve on a resident context (single use, like BundleAdjuster::Solve);
 * parameters stay on the device until mi_ba_context_writeback. */
mi_ba_status mi_ba_context_solve(mi_ba_context* ctx, mi_ba_summary* summary);
/* Copy the refined parameters back into the caller's problem arrays. */
mi_ba_status mi_ba_context_writeback(mi_ba_context* ctx);
/* Total cost 0.5*sum(rho) at the current parameters (geometric + semantic). */
mi_ba_status mi_ba_context_cost(mi_ba_context* ctx, double* cost);

/* --- multi-GPU LM (one process per GPU) ---------------------------------
 * Replaces the single-process Ceres solve with a point-sharded one (SURVEY
 * 8e): each rank creates its context from its own shard — all cameras and
 * images, the observations of its own points (point-major ranges) and its
 * own semantic image pairs — and joins a communicator before
 * mi_ba_context_solve.  Per LM iteration the camera-side normal-equation
 * blocks, the explicit reduced camera system S and the cost scalars are
 * summed over ranks; every rank then factors the same S and back-substitutes
 * its own points (exact Schur), or every Schur product of the implicit-Schur
 * PCG is summed as one nf-vector (ITERATIVE_SCHUR, the N > 1 default).
 * Sums go over the ranks whenever a reducer is installed, also at world 1
 * (a 1-rank communicator runs the multi-rank code path; tests/test_comm.py).
 *
 * Failure: every RCCL call is polled with a deadline ("comm_timeout_ms",
 * default 300 000): a collective or a communicator set-up that has not
 * completed by then, or that reports an asynchronous error
 * (ncclCommGetAsyncError), aborts the communicator (ncclCommAbort) and the
 * call returns MI_BA_ERR_HIP — a dead or diverged peer ends the solve
 * instead of hanging it.  After a failed set_comm the context remains a
 * single-rank context; after a failed collective every later one fails.
 *
 * mi_ba_comm_unique_id: RCCL unique id (ncclGetUniqueId) to be created on
 * rank 0 and broadcast by the caller (e.g. torch.distributed). */
#define MI_BA_COMM_ID_BYTES 128
mi_ba_status mi_ba_comm_unique_id(char id[MI_BA_COMM_ID_BYTES]);
/* Join rank `rank` of `world` over RCCL (xGMI on one node); non-blocking
 * set-up polled to the "comm_timeout_ms" deadline (set that key first). */
mi_ba_status mi_ba_context_set_comm(mi_ba_context* ctx, int32_t rank, int32_t world,
                                    const char id[MI_BA_COMM_ID_BYTES]);
/* Number of communicator set-ups still running on their helper threads (a
 * failed or timed-out set_comm ends its helper by the same deadline: the
 * helper stops polling, aborts the half-built communicator and exits). */
int32_t mi_ba_comm_pending_setups(void);
/* Alternative reducer for hosts without one GPU per rank: sums `n` doubles of
 * a host buffer in place across ranks (returns 0 on success).  Used by the
 * 1-GPU multi-rank rehearsal (gloo). */
typedef int32_t (*mi_ba_host_allreduce_fn)(double* data, int64_t n, void* user);
mi_ba_status mi_ba_context_set_host_reducer(mi_ba_context* ctx, int32_t rank, int32_t world,
                                            mi_ba_host_allreduce_fn fn, void* user);

/* Kernel-variant switches for in-process A/B measurement (key, value);
 * unknown keys return MI_BA_ERR_INVALID_ARGUMENT.  Keys:
 *   "comm_timeout_ms"       deadline of one RCCL collective / of set_comm (default
 *                           300000); a collective past it aborts the communicator
 *   "comm_stall_ms"         test hook: a kernel holds the stream this long ahead of
 *                           every RCCL collective (0 = off), as a missing peer would
 *   "jacobian_variant"      0 production; 1/4 row-staging passes, 9/10 no-store /
 *                           no-arithmetic roofline builds (11/12 the same of the
 *                           one-pass production shape), 20-22 store variants,
 *                           30-35 occupancy study (tools/ab_jacobian.py)
 *   "cholesky_panel"        0 recursive split, 64..4096 right-looking panel width
 *   "cholesky_gemm_update"  0 dsyrk / 1 dgemm trailing update
 *   "cholesky_own_diag"     6 one launch per panel for the diagonal block and the panel
 *                           solve (default; panels <= 512, else 2), 1 hand-written
 *                           diagonal-block factor (one column per step) + dtrsm, 2 the
 *                           same blocked by 4 (3: by 8) columns per step, 0 rocsolver_dpotrf
 *   "cholesky_rest_update"  trailing update after the look-ahead column: 3 dgemm per
 *                           1024-wide block column (default), 0 per 512, 1 dsyrk, 2 dgemmt
 *   "cholesky_rest_streams" those block columns dealt round-robin over this many
 *                           streams (1-4; default 2)
 *   "cholesky_rest_cumask" / "cholesky_rest_priority"  1: the extra streams created
 *                           with an all-CU mask / at the highest priority (measured
 *                           slower; default 0)
 *   "schur_pairs_variant"   0 explicit Schur pair kernel (default), 1-3 pipelined variants
 *   "semantic_variant"      6 flat pass (samples whose stencil provably stays on
 *                           the centre's outcome: J = 0) + deferred-sample pass
 *                           (default); 5 flat test + in-tile gather; 4, 3, 2
 *                           batched stencil with 4 / 2 / 1 parameters per step;
 *                           1 per-point FMA route; 0 per-point uncontracted
 *                           (all bitwise equal)
 *   "semantic_diag"         1: downloaded status is offset by +0x1000 for samples
 *                           the flat test deferred (variants 5, 6; diagnostic); 2:
 *                           also by +0x4000 for samples settled without the rasters
 *   "semantic_label_planes" 1 (default): the flat pass reads an 8-bit label index
 *                           plane and 8 x 8 tile depth ranges first (left off when the
 *                           rasters hold more than 256 distinct labels); 0 off
 *   "semantic_window_summary" 1: 3x3 window summaries of every raster pixel (the
 *                           default when the label planes are off); 0 off
 *   "linearize_warm_inputs" range mask of the reprojection kernel's inputs read into
 *                           the memory-side cache right before it (semantic contexts):
 *                           1 observations, 2 image ids, 4 point ids, 8 points;
 *                           default 15, 0 off
 *   "semantic_flat_coarse"  the flat pass's pixel box from a rotation and a translation
 *                           group of the stencil classes: 2 (default) with the camera
 *                           model's Jacobian at the centre, 1 with |A| bounded from the
 *                           radius, 3 the groups bounded apart; 0 per class
 *   "warm_workgroups"       workgroups of that read (default 2048; 0 one per CU)
 *   "linearize_overlap"     1 semantic kernel on a second stream beside the reprojection
 *                           kernel, 0 one stream (default)
 *   "cholesky_lookahead"    1 side-stream look-ahead (default) / 0 serial
 *   "cholesky_la_side_from" the look-ahead's dgemm (the next panel's block column)
 *                           on the side stream for panels starting at or after this
 *                           column (default 0: all but the first); -1: on the
 *                           caller's stream (bitwise equal)
 *   "schur_self_one_load"   1 (default): the Schur pair kernel's self tiles load each
 *                           Z row once; 0 twice (tools build; bitwise equal)
 *   "cholesky_solve"        2 sync-free triangular sweeps, one launch per direction
 *                           (default) / 1 hand-written blocked triangular sweeps /
 *                           0 recursive rocBLAS dtrsv + dgemv
 *   "cholesky_wait_ms"      bound of each in-launch flag wait of the factor and the
 *                           triangular sweeps, in wall-clock milliseconds (default
 *                           5000, at most 40000).  A wait that runs out makes the
 *                           solve return MI_BA_ERR_HIP (a hard error, never a
 *                           silently wrong factor)
 *   "cholesky_spin_log2"    0: no polling, so a wait on a flag not already set runs
 *                           out at once (the hook of the timeout test); any other
 *                           value (default 24): the time bound above */
mi_ba_status mi_ba_set_tuning(mi_ba_context* ctx, const char* key, int32_t value);

/* Dense Cholesky of a symmetric positive-definite n x n matrix with the
 * factorisation the exact Schur solver applies to the reduced camera system
 * (the replacement of the DENSE_SCHUR / SPARSE_SCHUR factorisation Ceres runs
 * inside BundleAdjuster::Solve, bundle_adjustment.cc:276-306), exposed for
 * parity tests and for callers that assemble their own S.  A: host, column-
 * major, lda = n; its lower triangle is read and overwritten with L (the
 * strict upper triangle is left as given).  b (nullable, host, n): on return
 * the solution of A x = b.  panel / lookahead / own_diag as the cholesky_*
 * tuning keys (panel 0 = recursive split).  *info = 0, or (panel > 0) the
 * 1-based column of the first pivot found not positive definite, (panel = 0)
 * a positive value (A unspecified in both cases).
 * Every call owns its stream, handles and workspace: concurrent calls from
 * several host threads share nothing. */
mi_ba_status mi_ba_dense_cholesky(int32_t device, int32_t n, double* A, double* b, int32_t panel, int32_t lookahead,
                                  int32_t own_diag, int32_t* info);
/* As mi_ba_dense_cholesky with the triangular-solve variant of the
 * "cholesky_solve" tuning key (2 sync-free sweeps = the default of
 * mi_ba_dense_cholesky, 1 per-block-column sweeps, 0 rocBLAS dtrsv/dgemv). */
mi_ba_status mi_ba_dense_cholesky_ex(int32_t device, int32_t n, double* A, double* b, int32_t panel,
                                     int32_t lookahead, int32_t own_diag, int32_t solve, int32_t* info);

/* Per-kernel HIP-event timing on the context's stream (enabled with
 * mi_ba_set_timing).  name: "reproj_jacobian", "semantic_jacobian", ... */
mi_ba_status mi_ba_set_timing(mi_ba_context* ctx, int32_t enabled);
mi_ba_status mi_ba_kernel_time(mi_ba_context* ctx, const char* name,
                               double* total_ms, int64_t* launches);
mi_ba_status mi_ba_reset_kernel_times(mi_ba_context* ctx);

#ifdef __cplusplus
}
#endif

#endif /* MI_BA_H_ */
