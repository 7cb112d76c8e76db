// colmap_amd/tiff.h — float32 TIFF raster loader for the semantic maps
// (header-only, host code).
//
//   MatrixFromTiff  <- matrixFromTiff (src/util/matrix_vis.h:130-176)
//   LoadSemanticMaps (ReadDepthAndSemanticMaps, src/optim/semantic_bundle_adjustment.cc:
//   1021-1068) is in semantic_bundle_adjustment.h.
//
// The reference loads through FreeImage, whose bitmaps are stored bottom-up,
// and writes matrix(height - 1 - i, j) = scanline i: the Eigen matrix is the
// raster in the file's natural top-down order (row y = image row y, column x
// = image column x).  MatrixFromTiff returns that matrix row-major
// ([y][x], y = 0 the first row in the file), the layout mi_ba_semantic takes.
// 32 bits per pixel only (matrix_vis.h:146-150), one sample per pixel, the
// bits read as an IEEE float32 as the reference's memcpy does.
//
// Supported: little/big-endian TIFF, strips or tiles, compression none (1),
// LZW (5), PackBits (32773) and — when COLMAP_AMD_TIFF_ZLIB is defined and
// the program links zlib — Deflate (8, 32946); predictor none (1),
// horizontal (2, on the 32-bit sample values) and floating point (3).
// Anything else throws std::runtime_error("Error loading depth map.") as the
// reference does for an unreadable file.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>


#ifdef COLMAP_AMD_TIFF_ZLIB
#include <zlib.h>
#endif

namespace colmap_amd {

namespace tiff {

[[noreturn]] inline void Fail(const std::string& why) {
  throw std::runtime_error("Error loading depth map. (" + why + ")");
}

struct File {
  std::vector<uint8_t> d;
  bool be = false;
  uint16_t U16(size_t o) const {
    if (o + 2 > d.size()) Fail("truncated");
    return be ? (uint16_t)(d[o] << 8 | d[o + 1]) : (uint16_t)(d[o] | d[o + 1] << 8);
  }
  uint32_t U32(size_t o) const {
    if (o + 4 > d.size()) Fail("truncated");
    return be ? ((uint32_t)d[o] << 24 | (uint32_t)d[o + 1] << 16 | (uint32_t)d[o + 2] << 8 | d[o + 3])
              : ((uint32_t)d[o] | (uint32_t)d[o + 1] << 8 | (uint32_t)d[o + 2] << 16 | (uint32_t)d[o + 3] << 24);
  }
};

// Values of one IFD entry (SHORT or LONG, inline or at an offset).
inline std::vector<uint32_t> EntryValues(const File& f, size_t e) {
  const uint16_t type = f.U16(e + 2);
  const uint32_t count = f.U32(e + 4);
  const size_t size = type == 3 ? 2 : type == 4 ? 4 : 0;
  if (size == 0) return {};
  const size_t base = (size * count <= 4) ? e + 8 : f.U32(e + 8);
  // bounds first: a hostile count must not size the allocation
  if ((uint64_t)base + (uint64_t)size * count > f.d.size()) Fail("truncated");
  std::vector<uint32_t> v(count);
  for (uint32_t k = 0; k < count; ++k) v[k] = size == 2 ? f.U16(base + 2 * k) : f.U32(base + 4 * k);
  return v;
}

// TIFF LZW (MSB-first codes, 9..12 bits, "early change").
inline std::vector<uint8_t> Lzw(const uint8_t* in, size_t n, size_t expect) {
  std::vector<uint8_t> out;
  out.reserve(expect);
  std::vector<std::vector<uint8_t>> dict;
  auto reset = [&]() {
    dict.assign(258, {});
    for (int k = 0; k < 256; ++k) dict[k] = {(uint8_t)k};
  };
  reset();
  size_t bitpos = 0;
  int width = 9;
  int prev = -1;
  while (true) {
    if (bitpos + width > 8 * n) break;
    uint32_t code = 0;
    for (int b = 0; b < width; ++b, ++bitpos) code = (code << 1) | ((in[bitpos >> 3] >> (7 - (bitpos & 7))) & 1u);
    if (code == 257) break;  // EOI
    if (code == 256) {       // Clear
      reset();
      width = 9;
      prev = -1;
      continue;
    }
    std::vector<uint8_t> entry;
    if (prev >= 0 && dict.size() >= 4096) Fail("bad LZW code");  // 12-bit table full without a Clear
    if (code < dict.size()) {
      entry = dict[code];
      if (prev >= 0) {
        std::vector<uint8_t> add = dict[prev];
        add.push_back(entry[0]);
        dict.push_back(add);
      }
    } else if (prev >= 0 && code == dict.size()) {
      entry = dict[prev];
      entry.push_back(entry[0]);
      dict.push_back(entry);
    } else {
      Fail("bad LZW code");
    }
    out.insert(out.end(), entry.begin(), entry.end());
    if (out.size() >= expect) break;  // the block's bytes are complete: no unbounded output
    prev = (int)code;
    if (dict.size() + 1 >= (1u << width) && width < 12) ++width;
  }
  return out;
}

inline std::vector<uint8_t> PackBits(const uint8_t* in, size_t n) {
  std::vector<uint8_t> out;
  size_t k = 0;
  while (k < n) {
    const int8_t h = (int8_t)in[k++];
    if (h >= 0) {
      const size_t c = (size_t)h + 1;
      if (k + c > n) Fail("PackBits");
      out.insert(out.end(), in + k, in + k + c);
      k += c;
    } else if (h != -128) {
      if (k >= n) Fail("PackBits");
      out.insert(out.end(), (size_t)(1 - h), in[k++]);
    }
  }
  return out;
}

inline std::vector<uint8_t> Inflate(const uint8_t* in, size_t n, size_t expect) {
#ifdef COLMAP_AMD_TIFF_ZLIB
  std::vector<uint8_t> out(expect);
  uLongf len = (uLongf)expect;
  if (uncompress(out.data(), &len, in, (uLong)n) != Z_OK) Fail("deflate");
  out.resize(len);
  return out;
#else
  (void)in; (void)n; (void)expect;
  Fail("Deflate TIFF needs COLMAP_AMD_TIFF_ZLIB and zlib");
#endif
}

// One decoded block (strip or tile) of `rows` rows of `cols` 32-bit samples
// in file byte order -> host floats, predictor undone.
inline void Unpredict(std::vector<uint8_t>& b, int predictor, bool be, size_t rows, size_t cols) {
  if (b.size() < rows * cols * 4) Fail("short block");
  if (predictor == 3) {
    // floating-point predictor: per row, bytes differenced, then stored most
    // significant byte plane first
    std::vector<uint8_t> tmp(cols * 4);
    for (size_t r = 0; r < rows; ++r) {
      uint8_t* row = b.data() + r * cols * 4;
      for (size_t k = 1; k < cols * 4; ++k) row[k] = (uint8_t)(row[k] + row[k - 1]);
      for (size_t c = 0; c < cols; ++c)
        for (int byte = 0; byte < 4; ++byte) tmp[4 * c + byte] = row[byte * cols + c];  // big-endian sample
      for (size_t c = 0; c < cols; ++c) {
        // to the file's byte order (converted to host below)
        if (!be) {
          for (int byte = 0; byte < 4; ++byte) row[4 * c + byte] = tmp[4 * c + 3 - byte];
        } else {
          for (int byte = 0; byte < 4; ++byte) row[4 * c + byte] = tmp[4 * c + byte];
        }
      }
    }
  } else if (predictor == 2) {
    for (size_t r = 0; r < rows; ++r) {
      uint8_t* row = b.data() + r * cols * 4;
      uint32_t prev = 0;
      for (size_t c = 0; c < cols; ++c) {
        uint32_t v;
        const uint8_t* p = row + 4 * c;
        v = be ? ((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3])
               : ((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
        v += prev;
        prev = v;
        uint8_t* q = row + 4 * c;
        if (be) { q[0] = v >> 24; q[1] = v >> 16; q[2] = v >> 8; q[3] = v; }
        else { q[0] = v; q[1] = v >> 8; q[2] = v >> 16; q[3] = v >> 24; }
      }
    }
  } else if (predictor != 1) {
    Fail("predictor");
  }
}

}  // namespace tiff

// matrixFromTiff (matrix_vis.h:130-176): row-major [height][width] float32.
inline std::vector<float> MatrixFromTiff(const std::string& path, int* height, int* width) {
  using namespace tiff;
  File f;
  {
    std::ifstream in(path, std::ios::binary);
    if (!in.is_open()) Fail("cannot open " + path);
    f.d.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
  }
  if (f.d.size() < 8) Fail("not a TIFF");
  if (f.d[0] == 'M' && f.d[1] == 'M') f.be = true;
  else if (!(f.d[0] == 'I' && f.d[1] == 'I')) Fail("not a TIFF");
  if (f.U16(2) != 42) Fail("not a classic TIFF");
  const size_t ifd = f.U32(4);
  const uint16_t ne = f.U16(ifd);
  std::unordered_map<uint16_t, std::vector<uint32_t>> tag;
  for (uint16_t k = 0; k < ne; ++k) {
    const size_t e = ifd + 2 + 12 * (size_t)k;
    tag[f.U16(e)] = EntryValues(f, e);
  }
  auto one = [&](uint16_t t, uint32_t dflt) {
    auto it = tag.find(t);
    return (it == tag.end() || it->second.empty()) ? dflt : it->second[0];
  };
  const uint32_t W = one(256, 0), H = one(257, 0);
  const uint32_t bps = one(258, 1), spp = one(277, 1), comp = one(259, 1), pred = one(317, 1);
  if (W == 0 || H == 0) Fail("size");
  if (bps * spp != 32) Fail("Probably not working with not float32 values.");  // matrix_vis.h:146-150
  if (spp != 1) Fail("samples per pixel");
  auto decode = [&](size_t off, size_t len, size_t expect) -> std::vector<uint8_t> {
    if (off + len > f.d.size()) Fail("block out of file");
    const uint8_t* p = f.d.data() + off;
    switch (comp) {
      case 1: return std::vector<uint8_t>(p, p + len);
      case 5: return Lzw(p, len, expect);
      case 32773: return PackBits(p, len);
      case 8:
      case 32946: return Inflate(p, len, expect);
      default: Fail("compression " + std::to_string(comp));
    }
  };
  auto to_float = [&](const uint8_t* p) {
    uint32_t v = f.be ? ((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3])
                      : ((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
    float x;
    std::memcpy(&x, &v, 4);
    return x;
  };
  if ((uint64_t)W * H > (1ull << 28)) Fail("size");  // 1 GB of float32 at most
  std::vector<float> out((size_t)W * H);
  if (tag.count(322)) {  // tiles
    const uint32_t tw = one(322, 0), th = one(323, 0);
    const auto& offs = tag[324];
    const auto& lens = tag[325];
    if (tw == 0 || th == 0) Fail("tile size");
    const uint32_t across = (W + tw - 1) / tw, down = (H + th - 1) / th;
    if (offs.size() < (size_t)across * down || lens.size() < offs.size()) Fail("tile table");
    for (uint32_t ty = 0; ty < down; ++ty)
      for (uint32_t tx = 0; tx < across; ++tx) {
        const size_t t = (size_t)ty * across + tx;
        std::vector<uint8_t> b = decode(offs[t], lens[t], (size_t)tw * th * 4);
        Unpredict(b, (int)pred, f.be, th, tw);
        for (uint32_t y = 0; y < th && ty * th + y < H; ++y)
          for (uint32_t x = 0; x < tw && tx * tw + x < W; ++x)
            out[(size_t)(ty * th + y) * W + tx * tw + x] = to_float(&b[((size_t)y * tw + x) * 4]);
      }
  } else {  // strips
    const uint32_t rps = std::min<uint32_t>(one(278, H), H);
    if (rps == 0) Fail("RowsPerStrip");
    const auto& offs = tag[273];
    const auto& lens = tag[279];
    const uint32_t nstrips = (H + rps - 1) / rps;
    if (offs.size() < nstrips || lens.size() < nstrips) Fail("strip table");
    for (uint32_t s = 0; s < nstrips; ++s) {
      const uint32_t rows = std::min(rps, H - s * rps);
      std::vector<uint8_t> b = decode(offs[s], lens[s], (size_t)rows * W * 4);
      Unpredict(b, (int)pred, f.be, rows, W);
      for (uint32_t y = 0; y < rows; ++y)
        for (uint32_t x = 0; x < W; ++x) out[(size_t)(s * rps + y) * W + x] = to_float(&b[((size_t)y * W + x) * 4]);
    }
  }
  *height = (int)H;
  *width = (int)W;
  return out;
}

}  // namespace colmap_amd

// LoadSemanticMaps (ReadDepthAndSemanticMaps) lives in semantic_bundle_adjustment.h;
// included here so existing callers keep working.
#include "semantic_bundle_adjustment.h"
