// colmap_amd/model_io.h — COLMAP sparse-model files for the facade's
// Reconstruction (header-only, host code).
//
//   ReadModel / ReadModelBinary / ReadModelText  <- Reconstruction::Read /
//       ReadBinary / ReadText (src/base/reconstruction.cc:733-760,
//       1525-1880): cameras, images (registered), points3D with tracks
//   WriteModelBinary / WriteModelText            <- Reconstruction::WriteBinary /
//       WriteText (reconstruction.cc:1882-2100); qvec written normalised,
//       text with 17 significant digits
//
// Formats: cameras.bin = u64 n; {u32 id, i32 model, u64 width, u64 height,
// f64 params[num_params(model)]}.  images.bin = u64 n; {u32 id, f64 qvec[4],
// f64 tvec[3], u32 camera_id, name '\0', u64 n2d; {f64 x, f64 y, u64
// point3D_id (max = none)}}.  points3D.bin = u64 n; {u64 id, f64 xyz[3], u8
// rgb[3], f64 error, u64 track_len; {u32 image_id, u32 point2D_idx}}.  All
// little-endian.  The text files hold the same fields, '#' comment lines,
// MODEL by name, POINT3D_ID -1 for none.  Errors throw std::runtime_error
// (the reference aborts through glog CHECK).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "reconstruction.h"

namespace colmap_amd {

namespace model_io {

// camera_models.h model ids / names / parameter counts (all COLMAP 3.8
// models; the BA path computes the first five).
struct ModelInfo {
  int id;
  const char* name;
  int num_params;
};
inline const ModelInfo* Models(int* n) {
  static const ModelInfo k[] = {{0, "SIMPLE_PINHOLE", 3},   {1, "PINHOLE", 4},
                                {2, "SIMPLE_RADIAL", 4},    {3, "RADIAL", 5},
                                {4, "OPENCV", 8},           {5, "OPENCV_FISHEYE", 8},
                                {6, "FULL_OPENCV", 12},     {7, "FOV", 5},
                                {8, "SIMPLE_RADIAL_FISHEYE", 4}, {9, "RADIAL_FISHEYE", 5},
                                {10, "THIN_PRISM_FISHEYE", 12}};
  *n = (int)(sizeof(k) / sizeof(k[0]));
  return k;
}
inline const ModelInfo& ModelById(int id) {
  int n;
  const ModelInfo* m = Models(&n);
  for (int k = 0; k < n; ++k)
    if (m[k].id == id) return m[k];
  throw std::runtime_error("unknown camera model id " + std::to_string(id));
}
inline const ModelInfo& ModelByName(const std::string& name) {
  int n;
  const ModelInfo* m = Models(&n);
  for (int k = 0; k < n; ++k)
    if (name == m[k].name) return m[k];
  throw std::runtime_error("unknown camera model " + name);
}

inline bool Exists(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  return f.good();
}
inline std::string Join(const std::string& a, const std::string& b) {
  return a.empty() || a.back() == '/' ? a + b : a + "/" + b;
}

class BinReader {
 public:
  explicit BinReader(const std::string& path) : f_(path, std::ios::binary) {
    if (!f_.is_open()) throw std::runtime_error("cannot open " + path);
    path_ = path;
  }
  template <typename T>
  T Get() {
    unsigned char b[sizeof(T)];
    if (!f_.read(reinterpret_cast<char*>(b), sizeof(T))) throw std::runtime_error("truncated " + path_);
    // little-endian file to host (x86-64 / gfx950 hosts are little-endian)
    T v;
    std::memcpy(&v, b, sizeof(T));
    return v;
  }
  std::string GetName() {
    std::string s;
    char c;
    while (true) {
      if (!f_.read(&c, 1)) throw std::runtime_error("truncated " + path_);
      if (c == '\0') break;
      s += c;
    }
    return s;
  }

 private:
  std::ifstream f_;
  std::string path_;
};

class BinWriter {
 public:
  explicit BinWriter(const std::string& path) : f_(path, std::ios::binary | std::ios::trunc) {
    if (!f_.is_open()) throw std::runtime_error("cannot open " + path);
  }
  template <typename T>
  void Put(T v) {
    f_.write(reinterpret_cast<const char*>(&v), sizeof(T));
  }
  void PutName(const std::string& s) { f_.write(s.c_str(), (std::streamsize)s.size() + 1); }

 private:
  std::ofstream f_;
};

inline void NormalizedQvec(const double q[4], double out[4]) {  // NormalizeQuaternion (pose.cc:82-91)
  const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n == 0) {
    out[0] = 1; out[1] = out[2] = out[3] = 0;
    return;
  }
  for (int k = 0; k < 4; ++k) out[k] = q[k] / n;
}

inline std::vector<std::string> Tokens(const std::string& line) {
  std::vector<std::string> out;
  std::istringstream is(line);
  std::string item;
  while (is >> item) out.push_back(item);
  return out;
}

inline bool DataLine(std::ifstream& f, std::string* line) {
  while (std::getline(f, *line)) {
    size_t a = line->find_first_not_of(" \t\r\n");
    if (a == std::string::npos) {
      line->clear();
      return true;  // an empty line (a points2D line of an image without points)
    }
    size_t b = line->find_last_not_of(" \t\r\n");
    *line = line->substr(a, b - a + 1);
    if ((*line)[0] == '#') continue;
    return true;
  }
  return false;
}

}  // namespace model_io

// Reconstruction::ReadBinary (reconstruction.cc:1756-1880)
inline void ReadModelBinary(const std::string& dir, Reconstruction* rec) {
  using namespace model_io;
  *rec = Reconstruction();
  {
    BinReader r(Join(dir, "cameras.bin"));
    const uint64_t n = r.Get<uint64_t>();
    for (uint64_t k = 0; k < n; ++k) {
      Camera c;
      c.camera_id = r.Get<uint32_t>();
      c.model_id = r.Get<int32_t>();
      c.width = r.Get<uint64_t>();
      c.height = r.Get<uint64_t>();
      c.params.resize(ModelById(c.model_id).num_params);
      for (double& v : c.params) v = r.Get<double>();
      rec->AddCamera(c);
    }
  }
  {
    BinReader r(Join(dir, "images.bin"));
    const uint64_t n = r.Get<uint64_t>();
    for (uint64_t k = 0; k < n; ++k) {
      Image im;
      im.image_id = r.Get<uint32_t>();
      for (double& v : im.qvec) v = r.Get<double>();
      for (double& v : im.tvec) v = r.Get<double>();
      im.camera_id = r.Get<uint32_t>();
      im.name = r.GetName();
      const uint64_t n2 = r.Get<uint64_t>();
      im.points2D.resize(n2);
      for (Point2D& p : im.points2D) {
        p.xy[0] = r.Get<double>();
        p.xy[1] = r.Get<double>();
        p.point3D_id = r.Get<uint64_t>();
      }
      im.registered = true;
      rec->AddImage(im);
    }
  }
  {
    BinReader r(Join(dir, "points3D.bin"));
    const uint64_t n = r.Get<uint64_t>();
    for (uint64_t k = 0; k < n; ++k) {
      const point3D_t id = r.Get<uint64_t>();
      Point3D p;
      for (double& v : p.xyz) v = r.Get<double>();
      for (uint8_t& v : p.color) v = r.Get<uint8_t>();
      p.error = r.Get<double>();
      const uint64_t len = r.Get<uint64_t>();
      p.track.resize(len);
      for (TrackElement& te : p.track) {
        te.image_id = r.Get<uint32_t>();
        te.point2D_idx = r.Get<uint32_t>();
      }
      rec->SetPoint3D(id, p);
    }
  }
}

// Reconstruction::ReadText (reconstruction.cc:1525-1754)
inline void ReadModelText(const std::string& dir, Reconstruction* rec) {
  using namespace model_io;
  *rec = Reconstruction();
  std::string line;
  {
    std::ifstream f(Join(dir, "cameras.txt"));
    if (!f.is_open()) throw std::runtime_error("cannot open " + Join(dir, "cameras.txt"));
    while (DataLine(f, &line)) {
      const auto t = Tokens(line);
      if (t.empty()) continue;
      if (t.size() < 4) throw std::runtime_error("cameras.txt: bad line");
      Camera c;
      c.camera_id = (camera_t)std::stoul(t[0]);
      c.model_id = ModelByName(t[1]).id;
      c.width = std::stoull(t[2]);
      c.height = std::stoull(t[3]);
      for (size_t k = 4; k < t.size(); ++k) c.params.push_back(std::stod(t[k]));
      if ((int)c.params.size() != ModelById(c.model_id).num_params)
        throw std::runtime_error("cameras.txt: parameter count");
      rec->AddCamera(c);
    }
  }
  {
    std::ifstream f(Join(dir, "images.txt"));
    if (!f.is_open()) throw std::runtime_error("cannot open " + Join(dir, "images.txt"));
    while (DataLine(f, &line)) {
      const auto t = Tokens(line);
      if (t.empty()) continue;
      if (t.size() < 10) throw std::runtime_error("images.txt: bad line");
      Image im;
      im.image_id = (image_t)std::stoul(t[0]);
      for (int k = 0; k < 4; ++k) im.qvec[k] = std::stod(t[1 + k]);
      for (int k = 0; k < 3; ++k) im.tvec[k] = std::stod(t[5 + k]);
      im.camera_id = (camera_t)std::stoul(t[8]);
      im.name = t[9];
      if (!DataLine(f, &line)) throw std::runtime_error("images.txt: missing POINTS2D line");
      const auto pts = Tokens(line);
      if (pts.size() % 3 != 0) throw std::runtime_error("images.txt: POINTS2D");
      for (size_t k = 0; k < pts.size(); k += 3) {
        Point2D p;
        p.xy[0] = std::stod(pts[k]);
        p.xy[1] = std::stod(pts[k + 1]);
        const long long id = std::stoll(pts[k + 2]);
        p.point3D_id = id < 0 ? kInvalidPoint3DId : (point3D_t)id;
        im.points2D.push_back(p);
      }
      im.registered = true;
      rec->AddImage(im);
    }
  }
  {
    std::ifstream f(Join(dir, "points3D.txt"));
    if (!f.is_open()) throw std::runtime_error("cannot open " + Join(dir, "points3D.txt"));
    while (DataLine(f, &line)) {
      const auto t = Tokens(line);
      if (t.empty()) continue;
      if (t.size() < 8 || (t.size() - 8) % 2 != 0) throw std::runtime_error("points3D.txt: bad line");
      Point3D p;
      const point3D_t id = std::stoull(t[0]);
      for (int k = 0; k < 3; ++k) p.xyz[k] = std::stod(t[1 + k]);
      for (int k = 0; k < 3; ++k) p.color[k] = (uint8_t)std::stoi(t[4 + k]);
      p.error = std::stod(t[7]);
      for (size_t k = 8; k < t.size(); k += 2)
        p.track.push_back(TrackElement{(image_t)std::stoul(t[k]), (point2D_t)std::stoul(t[k + 1])});
      rec->SetPoint3D(id, p);
    }
  }
}

// Reconstruction::Read (reconstruction.cc:733-745): binary if all three .bin
// files exist, else text.
inline void ReadModel(const std::string& dir, Reconstruction* rec) {
  using namespace model_io;
  if (Exists(Join(dir, "cameras.bin")) && Exists(Join(dir, "images.bin")) && Exists(Join(dir, "points3D.bin")))
    ReadModelBinary(dir, rec);
  else if (Exists(Join(dir, "cameras.txt")) && Exists(Join(dir, "images.txt")) && Exists(Join(dir, "points3D.txt")))
    ReadModelText(dir, rec);
  else
    throw std::runtime_error("cameras, images, points3D files do not exist at " + dir);
}

// Reconstruction::WriteBinary (reconstruction.cc:1994-2064); registered
// images only.
inline void WriteModelBinary(const std::string& dir, const Reconstruction& rec) {
  using namespace model_io;
  {
    BinWriter w(Join(dir, "cameras.bin"));
    w.Put<uint64_t>(rec.cameras.size());
    for (const auto& e : rec.cameras) {
      w.Put<uint32_t>(e.first);
      w.Put<int32_t>(e.second.model_id);
      w.Put<uint64_t>(e.second.width);
      w.Put<uint64_t>(e.second.height);
      for (double v : e.second.params) w.Put<double>(v);
    }
  }
  {
    BinWriter w(Join(dir, "images.bin"));
    uint64_t n = 0;
    for (const auto& e : rec.images) n += e.second.registered ? 1 : 0;
    w.Put<uint64_t>(n);
    for (const auto& e : rec.images) {
      if (!e.second.registered) continue;
      w.Put<uint32_t>(e.first);
      double q[4];
      NormalizedQvec(e.second.qvec, q);
      for (double v : q) w.Put<double>(v);
      for (double v : e.second.tvec) w.Put<double>(v);
      w.Put<uint32_t>(e.second.camera_id);
      w.PutName(e.second.name);
      w.Put<uint64_t>(e.second.points2D.size());
      for (const Point2D& p : e.second.points2D) {
        w.Put<double>(p.xy[0]);
        w.Put<double>(p.xy[1]);
        w.Put<uint64_t>(p.point3D_id);
      }
    }
  }
  {
    BinWriter w(Join(dir, "points3D.bin"));
    w.Put<uint64_t>(rec.points3D.size());
    for (const auto& e : rec.points3D) {
      w.Put<uint64_t>(e.first);
      for (double v : e.second.xyz) w.Put<double>(v);
      for (uint8_t v : e.second.color) w.Put<uint8_t>(v);
      w.Put<double>(e.second.error);
      w.Put<uint64_t>(e.second.track.size());
      for (const TrackElement& te : e.second.track) {
        w.Put<uint32_t>(te.image_id);
        w.Put<uint32_t>(te.point2D_idx);
      }
    }
  }
}

// Reconstruction::WriteText (reconstruction.cc:1882-1992), precision 17.
inline void WriteModelText(const std::string& dir, const Reconstruction& rec) {
  using namespace model_io;
  {
    std::ofstream f(Join(dir, "cameras.txt"), std::ios::trunc);
    if (!f.is_open()) throw std::runtime_error("cannot open " + Join(dir, "cameras.txt"));
    f.precision(17);
    f << "# Camera list with one line of data per camera:\n";
    f << "#   CAMERA_ID, MODEL, WIDTH, HEIGHT, PARAMS[]\n";
    f << "# Number of cameras: " << rec.cameras.size() << "\n";
    for (const auto& e : rec.cameras) {
      std::ostringstream line;
      line.precision(17);
      line << e.first << " " << ModelById(e.second.model_id).name << " " << e.second.width << " " << e.second.height;
      for (double v : e.second.params) line << " " << v;
      f << line.str() << "\n";
    }
  }
  {
    std::ofstream f(Join(dir, "images.txt"), std::ios::trunc);
    if (!f.is_open()) throw std::runtime_error("cannot open " + Join(dir, "images.txt"));
    f.precision(17);
    size_t n = 0, nobs = 0;
    for (const auto& e : rec.images)
      if (e.second.registered) {
        ++n;
        nobs += e.second.NumPoints3D();
      }
    f << "# Image list with two lines of data per image:\n";
    f << "#   IMAGE_ID, QW, QX, QY, QZ, TX, TY, TZ, CAMERA_ID, NAME\n";
    f << "#   POINTS2D[] as (X, Y, POINT3D_ID)\n";
    f << "# Number of images: " << n << ", mean observations per image: " << (n ? (double)nobs / n : 0.0) << "\n";
    for (const auto& e : rec.images) {
      if (!e.second.registered) continue;
      std::ostringstream line;
      line.precision(17);
      double q[4];
      NormalizedQvec(e.second.qvec, q);
      line << e.first << " " << q[0] << " " << q[1] << " " << q[2] << " " << q[3] << " " << e.second.tvec[0] << " "
           << e.second.tvec[1] << " " << e.second.tvec[2] << " " << e.second.camera_id << " " << e.second.name;
      f << line.str() << "\n";
      std::ostringstream pts;
      pts.precision(17);
      bool first = true;
      for (const Point2D& p : e.second.points2D) {
        if (!first) pts << " ";
        first = false;
        pts << p.xy[0] << " " << p.xy[1] << " ";
        if (p.HasPoint3D())
          pts << p.point3D_id;
        else
          pts << -1;
      }
      f << pts.str() << "\n";
    }
  }
  {
    std::ofstream f(Join(dir, "points3D.txt"), std::ios::trunc);
    if (!f.is_open()) throw std::runtime_error("cannot open " + Join(dir, "points3D.txt"));
    f.precision(17);
    size_t len = 0;
    for (const auto& e : rec.points3D) len += e.second.track.size();
    f << "# 3D point list with one line of data per point:\n";
    f << "#   POINT3D_ID, X, Y, Z, R, G, B, ERROR, TRACK[] as (IMAGE_ID, POINT2D_IDX)\n";
    f << "# Number of points: " << rec.points3D.size() << ", mean track length: "
      << (rec.points3D.empty() ? 0.0 : (double)len / rec.points3D.size()) << "\n";
    for (const auto& e : rec.points3D) {
      std::ostringstream line;
      line.precision(17);
      line << e.first << " " << e.second.xyz[0] << " " << e.second.xyz[1] << " " << e.second.xyz[2] << " "
           << (int)e.second.color[0] << " " << (int)e.second.color[1] << " " << (int)e.second.color[2] << " "
           << e.second.error;
      for (const TrackElement& te : e.second.track) line << " " << te.image_id << " " << te.point2D_idx;
      f << line.str() << "\n";
    }
  }
}

}  // namespace colmap_amd
