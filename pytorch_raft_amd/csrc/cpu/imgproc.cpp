// CPU image-processing runtime for the data pipeline (built into pytorch_raft_amd/_cpu.so).
//
// The reference leans on OpenCV for its host-side pipeline: cv2.resize(INTER_LINEAR) in the
// augmentors (`core/utils/augmentor.py:80-83,183-184`), cv2.imread/imwrite of 16-bit KITTI flow PNGs
// (`core/utils/frame_utils.py:102-120`) and cv2.remap in the warping demos (`demo_warp.py:59-73`).
// OpenCV is not part of this stack, so these are native C++ (OpenMP over rows), called through
// ctypes from pytorch_raft_amd/utils/imgproc.py:
//
//   raft_resize_linear_f32  bilinear resize with OpenCV INTER_LINEAR pixel-centre mapping
//                           (src = (dst + 0.5) * inv_scale - 0.5, replicated border)
//   raft_remap_linear_f32   backward warp: dst(p) = bilinear(src, map(p)), constant-0 border
//   raft_png_unfilter       PNG scanline un-filtering (None/Sub/Up/Average/Paeth) for the 8/16-bit
//                           PNG codec in pytorch_raft_amd/utils/png.py (zlib inflate stays in Python)
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>

extern "C" {

int raft_imgproc_version() { return 1; }

// src: (h, w, c) float32 row-major; dst: (oh, ow, c)
void raft_resize_linear_f32(const float* src, int h, int w, int c, float* dst, int oh, int ow,
                            double inv_sx, double inv_sy) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < oh; ++y) {
    double fy = (y + 0.5) * inv_sy - 0.5;
    int y0 = (int)std::floor(fy);
    float ay = (float)(fy - y0);
    int y1 = y0 + 1;
    if (y0 < 0) { y0 = 0; y1 = 0; ay = 0.f; }
    if (y1 >= h) { y1 = h - 1; if (y0 >= h) y0 = h - 1; if (y0 == y1) ay = 0.f; }
    const float* r0 = src + (size_t)y0 * w * c;
    const float* r1 = src + (size_t)y1 * w * c;
    float* out = dst + (size_t)y * ow * c;
    for (int x = 0; x < ow; ++x) {
      double fx = (x + 0.5) * inv_sx - 0.5;
      int x0 = (int)std::floor(fx);
      float ax = (float)(fx - x0);
      int x1 = x0 + 1;
      if (x0 < 0) { x0 = 0; x1 = 0; ax = 0.f; }
      if (x1 >= w) { x1 = w - 1; if (x0 >= w) x0 = w - 1; if (x0 == x1) ax = 0.f; }
      for (int k = 0; k < c; ++k) {
        float top = r0[x0 * c + k] + ax * (r0[x1 * c + k] - r0[x0 * c + k]);
        float bot = r1[x0 * c + k] + ax * (r1[x1 * c + k] - r1[x0 * c + k]);
        out[x * c + k] = top + ay * (bot - top);
      }
    }
  }
}

// map: (oh, ow, 2) absolute source coordinates (x, y)
void raft_remap_linear_f32(const float* src, int h, int w, int c, const float* map, float* dst,
                           int oh, int ow) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < oh; ++y) {
    for (int x = 0; x < ow; ++x) {
      const float mx = map[((size_t)y * ow + x) * 2];
      const float my = map[((size_t)y * ow + x) * 2 + 1];
      float* out = dst + ((size_t)y * ow + x) * c;
      if (!(std::isfinite(mx) && std::isfinite(my))) {
        for (int k = 0; k < c; ++k) out[k] = 0.f;
        continue;
      }
      // a coordinate beyond the +-1 pixel border samples only zeros; clamping first keeps the
      // float -> int conversion defined for any finite map value (UBSan float-cast-overflow)
      if (mx <= -1.f || my <= -1.f || mx >= (float)w || my >= (float)h) {
        for (int k = 0; k < c; ++k) out[k] = 0.f;
        continue;
      }
      const int x0 = (int)std::floor(mx), y0 = (int)std::floor(my);
      const float ax = mx - x0, ay = my - y0;
      float wts[4] = {(1 - ax) * (1 - ay), ax * (1 - ay), (1 - ax) * ay, ax * ay};
      int xs[4] = {x0, x0 + 1, x0, x0 + 1};
      int ys[4] = {y0, y0, y0 + 1, y0 + 1};
      for (int k = 0; k < c; ++k) out[k] = 0.f;
      for (int q = 0; q < 4; ++q) {
        if (xs[q] < 0 || xs[q] >= w || ys[q] < 0 || ys[q] >= h) continue;
        const float* s = src + ((size_t)ys[q] * w + xs[q]) * c;
        for (int k = 0; k < c; ++k) out[k] += wts[q] * s[k];
      }
    }
  }
}

static inline uint8_t paeth(int a, int b, int cc) {
  int p = a + b - cc;
  int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - cc);
  if (pa <= pb && pa <= pc) return (uint8_t)a;
  if (pb <= pc) return (uint8_t)b;
  return (uint8_t)cc;
}

// raw: rows * (1 + stride) inflated bytes (filter byte + scanline); out: rows * stride bytes.
// returns 0 on success, -1 on an unknown filter type.
int raft_png_unfilter(const uint8_t* raw, int rows, int stride, int bpp, uint8_t* out) {
  const uint8_t* prev = nullptr;
  for (int y = 0; y < rows; ++y) {
    const uint8_t* in = raw + (size_t)y * (stride + 1);
    const int ft = in[0];
    ++in;
    uint8_t* cur = out + (size_t)y * stride;
    switch (ft) {
      case 0: std::memcpy(cur, in, stride); break;
      case 1:
        for (int i = 0; i < stride; ++i) cur[i] = in[i] + (i >= bpp ? cur[i - bpp] : 0);
        break;
      case 2:
        for (int i = 0; i < stride; ++i) cur[i] = in[i] + (prev ? prev[i] : 0);
        break;
      case 3:
        for (int i = 0; i < stride; ++i) {
          int a = i >= bpp ? cur[i - bpp] : 0;
          int b = prev ? prev[i] : 0;
          cur[i] = in[i] + (uint8_t)((a + b) >> 1);
        }
        break;
      case 4:
        for (int i = 0; i < stride; ++i) {
          int a = i >= bpp ? cur[i - bpp] : 0;
          int b = prev ? prev[i] : 0;
          int cc = (prev && i >= bpp) ? prev[i - bpp] : 0;
          cur[i] = in[i] + paeth(a, b, cc);
        }
        break;
      default: return -1;
    }
    prev = cur;
  }
  return 0;
}

}  // extern "C"
