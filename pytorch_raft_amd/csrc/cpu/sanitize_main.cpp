// Sanitizer driver for the CPU image runtime (csrc/cpu/imgproc.cpp), built by
//   python -m pytorch_raft_amd.build --sanitize
// with -fsanitize=address,undefined,float-cast-overflow -fno-sanitize-recover=all and run by
// tests/test_sanitize.py.  Exercises every exported function on odd shapes, degenerate sizes
// (1-pixel images, 1-channel rows), extreme / non-finite remap coordinates and every PNG filter
// type, and checks the results against straightforward scalar references -- so an out-of-bounds
// access, an overflowing conversion or a wrong border rule fails the CPU test suite.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

extern "C" {
void raft_resize_linear_f32(const float*, int, int, int, float*, int, int, double, double);
void raft_remap_linear_f32(const float*, int, int, int, const float*, float*, int, int);
int raft_png_unfilter(const uint8_t*, int, int, int, uint8_t*);
}

static int g_fail = 0;
#define CHECK(c, ...)                                        \
  do {                                                       \
    if (!(c)) {                                              \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                     \
      std::fprintf(stderr, "\n");                            \
      ++g_fail;                                              \
    }                                                        \
  } while (0)

static uint32_t g_rng = 12345u;
static float frand() {
  g_rng = g_rng * 1664525u + 1013904223u;
  return (g_rng >> 8) * (1.0f / 16777216.0f);
}

static void test_resize() {
  const int shapes[][5] = {{1, 1, 1, 3, 4}, {7, 5, 3, 13, 2}, {16, 9, 2, 8, 17}, {3, 1, 4, 1, 9}};
  for (auto& s : shapes) {
    const int h = s[0], w = s[1], c = s[2], oh = s[3], ow = s[4];
    std::vector<float> src((size_t)h * w * c), dst((size_t)oh * ow * c, -1.f);
    for (auto& v : src) v = frand();
    raft_resize_linear_f32(src.data(), h, w, c, dst.data(), oh, ow, (double)w / ow, (double)h / oh);
    float lo = 1e9f, hi = -1e9f;
    for (float v : src) { lo = std::fmin(lo, v); hi = std::fmax(hi, v); }
    for (float v : dst) CHECK(std::isfinite(v) && v >= lo - 1e-5f && v <= hi + 1e-5f, "resize range %g", v);
  }
  // identity resize reproduces the input
  std::vector<float> a(5 * 7 * 2), b(a.size());
  for (auto& v : a) v = frand();
  raft_resize_linear_f32(a.data(), 5, 7, 2, b.data(), 5, 7, 1.0, 1.0);
  for (size_t i = 0; i < a.size(); ++i) CHECK(std::fabs(a[i] - b[i]) < 1e-6f, "identity %zu", i);
}

static void test_remap() {
  const int h = 5, w = 6, c = 3, oh = 4, ow = 9;
  std::vector<float> src((size_t)h * w * c);
  for (auto& v : src) v = frand();
  std::vector<float> map((size_t)oh * ow * 2), dst((size_t)oh * ow * c, -7.f);
  const float inf = std::numeric_limits<float>::infinity();
  const float special[] = {std::nanf(""), inf, -inf, 1e30f, -1e30f, -0.999f, (float)w - 1e-3f, 2.5f};
  for (int i = 0; i < oh * ow; ++i) {
    map[2 * i] = (i < 8) ? special[i] : frand() * (w + 4) - 2;
    map[2 * i + 1] = (i >= 8 && i < 16) ? special[i - 8] : frand() * (h + 4) - 2;
  }
  raft_remap_linear_f32(src.data(), h, w, c, map.data(), dst.data(), oh, ow);
  for (int i = 0; i < oh * ow; ++i) {
    const float mx = map[2 * i], my = map[2 * i + 1];
    for (int k = 0; k < c; ++k) {
      float ref = 0.f;
      if (std::isfinite(mx) && std::isfinite(my) && std::fabs(mx) < 1e6f && std::fabs(my) < 1e6f) {
        const int x0 = (int)std::floor(mx), y0 = (int)std::floor(my);
        const float ax = mx - x0, ay = my - y0;
        for (int q = 0; q < 4; ++q) {
          const int xx = x0 + (q & 1), yy = y0 + (q >> 1);
          const float wt = ((q & 1) ? ax : 1 - ax) * ((q >> 1) ? ay : 1 - ay);
          if (xx >= 0 && xx < w && yy >= 0 && yy < h) ref += wt * src[((size_t)yy * w + xx) * c + k];
        }
      }
      const float got = dst[(size_t)i * c + k];
      CHECK(std::isfinite(got) && std::fabs(got - ref) < 1e-5f, "remap %d/%d got %g ref %g", i, k, got, ref);
    }
  }
}

static void test_png() {
  const int rows = 5, stride = 11, bpp = 3;
  std::vector<uint8_t> raw((size_t)rows * (stride + 1)), out((size_t)rows * stride);
  for (auto& v : raw) v = (uint8_t)(frand() * 256);
  for (int y = 0; y < rows; ++y) raw[(size_t)y * (stride + 1)] = (uint8_t)y;  // filters 0..4
  CHECK(raft_png_unfilter(raw.data(), rows, stride, bpp, out.data()) == 0, "unfilter rc");
  // scalar re-implementation
  std::vector<uint8_t> ref(out.size());
  for (int y = 0; y < rows; ++y)
    for (int i = 0; i < stride; ++i) {
      const int v = raw[(size_t)y * (stride + 1) + 1 + i];
      const int a = i >= bpp ? ref[(size_t)y * stride + i - bpp] : 0;
      const int b = y ? ref[(size_t)(y - 1) * stride + i] : 0;
      const int cc = (y && i >= bpp) ? ref[(size_t)(y - 1) * stride + i - bpp] : 0;
      int p = 0;
      switch (y) {
        case 0: p = 0; break;
        case 1: p = a; break;
        case 2: p = b; break;
        case 3: p = (a + b) >> 1; break;
        default: {
          const int pp = a + b - cc, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - cc);
          p = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc);
        }
      }
      ref[(size_t)y * stride + i] = (uint8_t)(v + p);
    }
  for (size_t i = 0; i < out.size(); ++i) CHECK(out[i] == ref[i], "png byte %zu", i);
  raw[0] = 9;  // unknown filter type is rejected
  CHECK(raft_png_unfilter(raw.data(), rows, stride, bpp, out.data()) == -1, "bad filter accepted");
  // a single 1-byte row
  uint8_t one_raw[2] = {1, 200}, one_out[1] = {0};
  CHECK(raft_png_unfilter(one_raw, 1, 1, 1, one_out) == 0 && one_out[0] == 200, "1-byte row");
}

int main() {
  test_resize();
  test_remap();
  test_png();
  if (g_fail) {
    std::fprintf(stderr, "%d failures\n", g_fail);
    return 1;
  }
  std::printf("imgproc sanitize: ok\n");
  return 0;
}
