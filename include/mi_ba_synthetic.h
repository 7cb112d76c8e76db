/*
 * mi_ba_synthetic.h — synthetic BA scenes (benchmark / test fixture tool).
 *
 * Restates the reference's test fixture GenerateReconstruction
 * (src/optim/bundle_adjustment_test.cc:111-184): std::mt19937 seeded with
 * SetPRNGSeed(seed) and RandomReal = std::uniform_real_distribution<double>
 * (src/util/random.h:99-107, random.cc:38-42); points ~ U[-1,1]^3; one camera
 * per image with f = 1.2 * image_size and principal point at the centre;
 * tvec = (U(-1,1), U(-1,1), 10); observations = exact projection + U(-2,2)
 * noise.  track_length = 0 reproduces the reference (every point in every
 * image, identity rotations); track_length = L > 0 is the build's scaled
 * variant: each point seen by L distinct images,
 * small random rotations.  Rendering produces the semantic inputs: a
 * labelled plane Z = plane_z with label (floor(X/cell)+floor(Y/cell)) mod 8.
 */
#ifndef MI_BA_SYNTHETIC_H_
#define MI_BA_SYNTHETIC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mi_ba_synth_config {
  int32_t camera_model;   /* MI_BA_* */
  int32_t num_images;
  int64_t num_points;
  int32_t track_length;   /* 0 = every point in every image (reference) */
  int32_t image_size;     /* width = height, reference 1000 */
  double focal_factor;    /* f = focal_factor * image_size, reference 1.2 */
  double extra[4];        /* extra (distortion) params of the model */
  double rotation_range;  /* axis-angle components ~ U(-r, r); 0 = identity */
  double noise;           /* U(-noise, noise) px, reference 2 */
  uint32_t seed;          /* reference 0 */
} mi_ba_synth_config;

int64_t mi_ba_synth_num_obs(const mi_ba_synth_config* cfg);

/* Arrays sized: camera_params [num_images][num_params], qvec [I][4],
 * tvec [I][3], image_camera [I], xyz [P][3], obs_* [num_obs]. */
int32_t mi_ba_synth_generate(const mi_ba_synth_config* cfg, double* camera_params, double* qvec,
                             double* tvec, int32_t* image_camera, double* xyz, double* obs_xy,
                             int32_t* obs_image, int32_t* obs_point);

/* Depth (camera z) and label rasters [num_images][H][W] of the plane
 * Z = plane_z seen from each image (0 depth where the ray misses). */
int32_t mi_ba_synth_render(int32_t camera_model, int32_t num_images, const double* camera_params,
                           const double* qvec, const double* tvec, const int32_t* image_camera,
                           int32_t height, int32_t width, double plane_z, double cell, float* depth,
                           float* label);

#ifdef __cplusplus
}
#endif

#endif /* MI_BA_SYNTHETIC_H_ */
