// colmap_amd/reconstruction.h — the facade's Reconstruction (the subset of
// colmap::Reconstruction, src/base/reconstruction.{h,cc}, that bundle
// adjustment, the model files and the controllers touch): cameras, images
// with their registration order, points with tracks, observation edits and
// the two post-BA filters on the MI355X.  Header-only; link against
// libmi_ba.so.  Included by bundle_adjustment.h and model_io.h.
#pragma once

#include <algorithm>
#include <cstdint>
#include <limits>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../mi_ba.h"

namespace colmap_amd {

typedef uint32_t camera_t;
typedef uint32_t image_t;
typedef uint64_t point3D_t;
typedef uint32_t point2D_t;
const point3D_t kInvalidPoint3DId = std::numeric_limits<point3D_t>::max();

// ---------------------------------------------------------------------------
// Minimal Reconstruction (the parts BundleAdjuster touches).
// ---------------------------------------------------------------------------
struct Camera {
  camera_t camera_id = 0;
  int model_id = MI_BA_SIMPLE_RADIAL;
  uint64_t width = 0, height = 0;
  std::vector<double> params;
  double* ParamsData() { return params.data(); }
  int ModelId() const { return model_id; }
  camera_t CameraId() const { return camera_id; }
};

struct Point2D {
  double xy[2] = {0, 0};
  point3D_t point3D_id = kInvalidPoint3DId;
  bool HasPoint3D() const { return point3D_id != kInvalidPoint3DId; }
};

struct TrackElement {
  image_t image_id;
  point2D_t point2D_idx;
};

struct Image {
  image_t image_id = 0;
  camera_t camera_id = 0;
  std::string name;
  double qvec[4] = {1, 0, 0, 0};
  double tvec[3] = {0, 0, 0};
  std::vector<Point2D> points2D;
  bool registered = true;
  bool IsRegistered() const { return registered; }
  image_t ImageId() const { return image_id; }
  camera_t CameraId() const { return camera_id; }
  const std::string& Name() const { return name; }
  size_t NumPoints3D() const {
    return (size_t)std::count_if(points2D.begin(), points2D.end(), [](const Point2D& p) { return p.HasPoint3D(); });
  }
};

struct Point3D {
  double xyz[3] = {0, 0, 0};
  uint8_t color[3] = {0, 0, 0};
  double error = -1.0;
  std::vector<TrackElement> track;
};

class Reconstruction {
 public:
  std::map<camera_t, Camera> cameras;
  std::map<image_t, Image> images;
  std::map<point3D_t, Point3D> points3D;

  Camera& GetCamera(camera_t id) { return cameras.at(id); }
  Image& GetImage(image_t id) { return images.at(id); }
  Point3D& GetPoint3D(point3D_t id) { return points3D.at(id); }
  const Image& GetImage(image_t id) const { return images.at(id); }
  const Point3D& GetPoint3D(point3D_t id) const { return points3D.at(id); }

  void AddCamera(const Camera& c) { cameras[c.camera_id] = c; }
  // A registered image joins the registration order (reg_image_ids_) when it
  // is first added: the model readers add images in file order, as
  // ReadImagesBinary / ReadImagesText register them (reconstruction.cc:
  // 1599-1600,1826-1827).
  void AddImage(const Image& im) {
    const bool known = images.count(im.image_id) != 0;
    images[im.image_id] = im;
    if (im.registered && (!known || !InRegOrder(im.image_id))) reg_image_ids_.push_back(im.image_id);
  }
  // Reconstruction::RegisterImage / DeRegisterImage (reconstruction.cc:296-320)
  void RegisterImage(image_t id) {
    Image& im = images.at(id);
    if (!im.registered || !InRegOrder(id)) {
      im.registered = true;
      if (!InRegOrder(id)) reg_image_ids_.push_back(id);
    }
  }
  void DeRegisterImage(image_t id) {
    Image& im = images.at(id);
    for (point2D_t k = 0; k < (point2D_t)im.points2D.size(); ++k)
      if (images.at(id).points2D[k].HasPoint3D()) DeleteObservation(id, k);
    images.at(id).registered = false;
    reg_image_ids_.erase(std::remove(reg_image_ids_.begin(), reg_image_ids_.end(), id), reg_image_ids_.end());
  }
  // Reconstruction::RegImageIds: registered images in registration order.
  // Images whose `registered` flag was set directly (not through
  // RegisterImage / AddImage) follow in image-id order; cleared flags drop out.
  std::vector<image_t> RegImageIds() const {
    std::vector<image_t> ids;
    for (const image_t id : reg_image_ids_) {
      auto it = images.find(id);
      if (it != images.end() && it->second.registered) ids.push_back(id);
    }
    for (const auto& e : images)
      if (e.second.registered && !InRegOrder(e.first)) ids.push_back(e.first);
    return ids;
  }
  point3D_t AddPoint3D(const double xyz[3]) {
    const point3D_t id = ++num_added_points3D_;  // 1-based like COLMAP
    Point3D p;
    std::copy(xyz, xyz + 3, p.xyz);
    points3D[id] = p;
    return id;
  }
  // A point with a given id (model readers); later AddPoint3D ids continue after it.
  void SetPoint3D(point3D_t id, const Point3D& p) {
    points3D[id] = p;
    num_added_points3D_ = std::max(num_added_points3D_, id);
  }
  void AddObservation(point3D_t point3D_id, const TrackElement& te) {
    images.at(te.image_id).points2D.at(te.point2D_idx).point3D_id = point3D_id;
    points3D.at(point3D_id).track.push_back(te);
  }
  // Reconstruction::DeleteObservation (reconstruction.cc:257-277): a track
  // of length <= 2 takes its point with it.
  void DeleteObservation(image_t image_id, point2D_t point2D_idx) {
    Point2D& p2 = images.at(image_id).points2D.at(point2D_idx);
    auto& tr = points3D.at(p2.point3D_id).track;
    if (tr.size() <= 2) {
      DeletePoint3D(p2.point3D_id);
      return;
    }
    tr.erase(std::remove_if(tr.begin(), tr.end(),
                            [&](const TrackElement& t) { return t.image_id == image_id && t.point2D_idx == point2D_idx; }),
             tr.end());
    p2.point3D_id = kInvalidPoint3DId;
  }
  void DeletePoint3D(point3D_t id) {
    for (const TrackElement& te : points3D.at(id).track)
      images.at(te.image_id).points2D.at(te.point2D_idx).point3D_id = kInvalidPoint3DId;
    points3D.erase(id);
  }

  // Reconstruction::FilterPoints3DWithLargeReprojectionError
  // (reconstruction.cc:1472-1525) on the GPU (mi_ba_filter_points3d): the
  // given points' track elements are flattened in Track order, their errors
  // evaluated and the decisions applied here.  Returns the number of
  // observations filtered.
  size_t FilterPoints3DWithLargeReprojectionError(double max_reproj_error,
                                                  const std::unordered_set<point3D_t>& point3D_ids,
                                                  int device = 0);

  // Reconstruction::FilterObservationsWithNegativeDepth (reconstruction.cc:
  // 647-665): the depth test of every observation of the registered images
  // on the GPU (mi_ba_positive_depth), then the reference's deletions in
  // image / point2D order (registered images in registration order,
  // RegImageIds).  Returns the
  // number of observations deleted.
  size_t FilterObservationsWithNegativeDepth(int device = 0);

 private:
  bool InRegOrder(image_t id) const {
    return std::find(reg_image_ids_.begin(), reg_image_ids_.end(), id) != reg_image_ids_.end();
  }
  point3D_t num_added_points3D_ = 0;
  std::vector<image_t> reg_image_ids_;
};

namespace internal {

inline void ThrowStatus(mi_ba_status st, const char* what) {
  const std::string msg = std::string(what) + ": " + mi_ba_status_string(st);
  switch (st) {
    case MI_BA_OK: return;
    case MI_BA_ERR_INVALID_ARGUMENT: throw std::invalid_argument(msg);
    case MI_BA_ERR_UNSUPPORTED: throw std::domain_error(msg);
    case MI_BA_ERR_STATE: throw std::logic_error(msg);
    default: throw std::runtime_error(msg);
  }
}

}  // namespace internal

inline size_t Reconstruction::FilterPoints3DWithLargeReprojectionError(
    double max_reproj_error, const std::unordered_set<point3D_t>& point3D_ids, int device) {
  std::unordered_map<camera_t, int32_t> cidx;
  std::unordered_map<image_t, int32_t> iidx;
  std::vector<camera_t> cam_ids;
  std::vector<image_t> img_ids;
  std::vector<point3D_t> pt_ids;
  std::vector<double> params, qv, tv, xyz, obs_xy;
  std::vector<int32_t> models, image_camera, obs_image, obs_point;
  std::vector<TrackElement> obs_te;
  for (const auto& c : cameras) {
    cidx[c.first] = (int32_t)cam_ids.size();
    cam_ids.push_back(c.first);
    models.push_back(c.second.model_id);
    params.insert(params.end(), c.second.params.begin(), c.second.params.end());
  }
  for (const auto& im : images) {
    iidx[im.first] = (int32_t)img_ids.size();
    img_ids.push_back(im.first);
    qv.insert(qv.end(), im.second.qvec, im.second.qvec + 4);
    tv.insert(tv.end(), im.second.tvec, im.second.tvec + 3);
    image_camera.push_back(cidx.at(im.second.camera_id));
  }
  for (const point3D_t id : point3D_ids) {
    auto it = points3D.find(id);
    if (it == points3D.end()) continue;  // ExistsPoint3D (:1481-1483)
    const int32_t p = (int32_t)pt_ids.size();
    pt_ids.push_back(id);
    xyz.insert(xyz.end(), it->second.xyz, it->second.xyz + 3);
    for (const TrackElement& te : it->second.track) {
      const Point2D& p2 = images.at(te.image_id).points2D.at(te.point2D_idx);
      obs_xy.push_back(p2.xy[0]);
      obs_xy.push_back(p2.xy[1]);
      obs_image.push_back(iidx.at(te.image_id));
      obs_point.push_back(p);
      obs_te.push_back(te);
    }
  }
  mi_ba_problem pr{};
  pr.camera_model = models.empty() ? MI_BA_SIMPLE_RADIAL : models[0];
  pr.camera_model_ids = models.data();
  pr.num_cameras = (int32_t)cam_ids.size();
  pr.camera_params = params.data();
  pr.num_images = (int32_t)img_ids.size();
  pr.qvec = qv.data();
  pr.tvec = tv.data();
  pr.image_camera = image_camera.data();
  pr.num_points = (int64_t)pt_ids.size();
  pr.xyz = xyz.data();
  pr.num_obs = (int64_t)obs_image.size();
  pr.obs_xy = obs_xy.data();
  pr.obs_image = obs_image.data();
  pr.obs_point = obs_point.data();
  std::vector<uint8_t> obs_keep(obs_image.size()), point_keep(pt_ids.size());
  std::vector<double> err(pt_ids.size());
  for (size_t p = 0; p < pt_ids.size(); ++p) err[p] = points3D.at(pt_ids[p]).error;
  int64_t num_filtered = 0;
  internal::ThrowStatus(mi_ba_filter_points3d(&pr, max_reproj_error, nullptr, device, obs_keep.data(),
                                              point_keep.data(), err.data(), &num_filtered),
                        "FilterPoints3DWithLargeReprojectionError");
  for (size_t k = 0; k < obs_te.size(); ++k)
    if (point_keep[obs_point[k]] && !obs_keep[k]) DeleteObservation(obs_te[k].image_id, obs_te[k].point2D_idx);
  for (size_t p = 0; p < pt_ids.size(); ++p) {
    if (!point_keep[p]) DeletePoint3D(pt_ids[p]);
    else points3D.at(pt_ids[p]).error = err[p];
  }
  return (size_t)num_filtered;
}

inline size_t Reconstruction::FilterObservationsWithNegativeDepth(int device) {
  std::unordered_map<camera_t, int32_t> cidx;
  std::vector<double> params, qv, tv, xyz, obs_xy;
  std::vector<int32_t> models, image_camera, obs_image, obs_point;
  std::vector<uint8_t> reg;
  std::vector<std::pair<image_t, point2D_t>> obs_ref;
  std::unordered_map<point3D_t, int32_t> pidx;
  for (const auto& c : cameras) {
    cidx[c.first] = (int32_t)models.size();
    models.push_back(c.second.model_id);
    params.insert(params.end(), c.second.params.begin(), c.second.params.end());
  }
  for (const auto& p : points3D) {
    pidx[p.first] = (int32_t)(xyz.size() / 3);
    xyz.insert(xyz.end(), p.second.xyz, p.second.xyz + 3);
  }
  std::unordered_map<image_t, int32_t> iidx;
  for (const auto& im : images) {
    iidx[im.first] = (int32_t)image_camera.size();
    qv.insert(qv.end(), im.second.qvec, im.second.qvec + 4);
    tv.insert(tv.end(), im.second.tvec, im.second.tvec + 3);
    image_camera.push_back(cidx.at(im.second.camera_id));
    reg.push_back(im.second.IsRegistered() ? 1 : 0);
  }
  // reconstruction.cc:649: for (image_id : reg_image_ids_)
  for (const image_t id : RegImageIds()) {
    const Image& im = images.at(id);
    for (point2D_t k = 0; k < (point2D_t)im.points2D.size(); ++k) {
      const Point2D& p2 = im.points2D[k];
      if (!p2.HasPoint3D()) continue;
      obs_xy.push_back(p2.xy[0]);
      obs_xy.push_back(p2.xy[1]);
      obs_image.push_back(iidx.at(id));
      obs_point.push_back(pidx.at(p2.point3D_id));
      obs_ref.emplace_back(id, k);
    }
  }
  if (obs_ref.empty()) return 0;
  mi_ba_problem pr{};
  pr.camera_model = models.empty() ? MI_BA_SIMPLE_RADIAL : models[0];
  pr.camera_model_ids = models.data();
  pr.num_cameras = (int32_t)models.size();
  pr.camera_params = params.data();
  pr.num_images = (int32_t)image_camera.size();
  pr.qvec = qv.data();
  pr.tvec = tv.data();
  pr.image_camera = image_camera.data();
  pr.num_points = (int64_t)(xyz.size() / 3);
  pr.xyz = xyz.data();
  pr.num_obs = (int64_t)obs_image.size();
  pr.obs_xy = obs_xy.data();
  pr.obs_image = obs_image.data();
  pr.obs_point = obs_point.data();
  std::vector<uint8_t> keep(obs_ref.size());
  int64_t negative = 0;
  internal::ThrowStatus(mi_ba_positive_depth(&pr, reg.data(), device, keep.data(), &negative),
                        "FilterObservationsWithNegativeDepth");
  // the reference's deletions, in order: an observation whose point an
  // earlier deletion already removed is no longer counted (HasPoint3D)
  size_t num_filtered = 0;
  for (size_t k = 0; k < obs_ref.size(); ++k) {
    if (keep[k]) continue;
    if (!images.at(obs_ref[k].first).points2D.at(obs_ref[k].second).HasPoint3D()) continue;
    DeleteObservation(obs_ref[k].first, obs_ref[k].second);
    ++num_filtered;
  }
  return num_filtered;
}

}  // namespace colmap_amd
