// Torch operator registration for the pytorch_raft_amd gfx950 kernels.
//
// Every op validates device / dtype / contiguity / shape on the host BEFORE launching (a faulting
// kernel can reset the whole node), then calls the raw launchers in kernels/*.hip on the current
// HIP stream.  Ops are exposed as torch.ops.raft_amd.<name> (TORCH_LIBRARY), so the library needs
// no Python C-API and is loaded with torch.ops.load_library.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "kernels/launchers.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda_f32(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32, got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

struct Levels {
  std::vector<float*> ptr;
  std::vector<int> h, w;
};

Levels levels_of(const std::vector<Tensor>& lv, int64_t planes_expected, const char* name) {
  TORCH_CHECK(!lv.empty() && lv.size() <= 4, name, ": 1..4 levels required");
  Levels L;
  for (const auto& t : lv) {
    check_cuda_f32(t, name);
    TORCH_CHECK(t.dim() == 4, name, " levels must be (B, N, h, w)");
    TORCH_CHECK(t.size(0) * t.size(1) == planes_expected, name, " plane count mismatch");
    L.ptr.push_back(t.data_ptr<float>());
    L.h.push_back((int)t.size(2));
    L.w.push_back((int)t.size(3));
  }
  for (size_t l = 1; l < lv.size(); ++l)
    TORCH_CHECK(L.h[l] == L.h[l - 1] / 2 && L.w[l] == L.w[l - 1] / 2, name,
                " level sizes must follow floor(prev/2)");
  return L;
}

// ------------------------------------------------------------------ all-pairs correlation
std::vector<Tensor> corr_build(const Tensor& f1, const Tensor& f2, int64_t levels) {
  check_cuda_f32(f1, "fmap1");
  check_cuda_f32(f2, "fmap2");
  TORCH_CHECK(f1.dim() == 4 && f1.sizes() == f2.sizes(), "fmap1/fmap2 must be equal (B,C,H,W)");
  TORCH_CHECK(levels >= 1 && levels <= 4, "levels must be 1..4");
  c10::DeviceGuard g(f1.device());
  const int64_t B = f1.size(0), C = f1.size(1), H = f1.size(2), W = f1.size(3);
  const int64_t N = H * W;
  std::vector<Tensor> out;
  std::vector<float*> ptr;
  std::vector<int> hs, ws;
  int64_t h = H, w = W;
  for (int64_t l = 0; l < levels; ++l) {
    TORCH_CHECK(h >= 1 && w >= 1, "feature map too small for ", levels, " pyramid levels");
    out.push_back(at::empty({B, N, h, w}, f1.options()));
    ptr.push_back(out.back().data_ptr<float>());
    hs.push_back((int)h);
    ws.push_back((int)w);
    h /= 2;
    w /= 2;
  }
  launch_corr_build(f1.data_ptr<float>(), f2.data_ptr<float>(), ptr.data(), hs.data(), ws.data(),
                    (int)B, (int)C, (int)H, (int)W, (int)levels, cur_stream());
  return out;
}

// bf16 fmaps in NHWC memory, (B,H,W,C) contiguous (the channels_last encoder outputs, permuted)
std::vector<Tensor> corr_build_bf16(const Tensor& f1, const Tensor& f2, int64_t levels,
                                    bool pyr_bf16) {
  TORCH_CHECK(f1.is_cuda() && f2.is_cuda() && f1.scalar_type() == at::kBFloat16 &&
                  f2.scalar_type() == at::kBFloat16 && f1.is_contiguous() && f2.is_contiguous(),
              "fmaps must be contiguous bf16 (B,H,W,C) GPU tensors");
  TORCH_CHECK(f1.dim() == 4 && f1.sizes() == f2.sizes(), "fmap1/fmap2 must be equal (B,H,W,C)");
  TORCH_CHECK(levels >= 1 && levels <= 4, "levels must be 1..4");
  const int64_t B = f1.size(0), H = f1.size(1), W = f1.size(2), C = f1.size(3);
  TORCH_CHECK(C % 16 == 0 && C > 0, "channels must be a multiple of 16");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(f1.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(f2.data_ptr()) & 15) == 0,
              "fmaps must be 16-B aligned");
  c10::DeviceGuard g(f1.device());
  const int64_t N = H * W;
  std::vector<Tensor> out;
  std::vector<void*> ptr;
  std::vector<int> hs, ws;
  int64_t h = H, w = W;
  auto fopt = f1.options().dtype(pyr_bf16 ? at::kBFloat16 : at::kFloat);
  for (int64_t l = 0; l < levels; ++l) {
    TORCH_CHECK(h >= 1 && w >= 1, "feature map too small for ", levels, " pyramid levels");
    out.push_back(at::empty({B, N, h, w}, fopt));
    ptr.push_back(out.back().data_ptr());
    hs.push_back((int)h);
    ws.push_back((int)w);
    h /= 2;
    w /= 2;
  }
  launch_corr_build_bf16(reinterpret_cast<const uint16_t*>(f1.data_ptr()),
                         reinterpret_cast<const uint16_t*>(f2.data_ptr()), ptr.data(), hs.data(),
                         ws.data(), (int)B, (int)C, (int)H, (int)W, (int)levels, pyr_bf16,
                         cur_stream());
  return out;
}

Tensor corr_lookup_fwd(const std::vector<Tensor>& pyr, const Tensor& coords, int64_t radius) {
  check_cuda_f32(coords, "coords");
  TORCH_CHECK(coords.dim() == 4 && coords.size(1) == 2, "coords must be (B,2,H,W)");
  TORCH_CHECK(radius == 3 || radius == 4, "radius must be 3 or 4");
  c10::DeviceGuard g(coords.device());
  const int64_t B = coords.size(0), H = coords.size(2), W = coords.size(3);
  Levels L = levels_of(pyr, B * H * W, "pyramid");
  TORCH_CHECK(L.h[0] == H && L.w[0] == W, "pyramid level 0 must match coords grid");
  const int64_t D = 2 * radius + 1;
  const int levels = (int)pyr.size();
  const int64_t N = H * W, Ct = levels * D * D;
  Tensor out = at::empty({B, Ct, H, W}, coords.options());
  std::vector<const float*> cp(L.ptr.begin(), L.ptr.end());
  TORCH_CHECK(launch_corr_lookup_fwd(cp.data(), L.h.data(), L.w.data(), levels,
                                     coords.data_ptr<float>(), out.data_ptr<float>(), 0, Ct * N, 1,
                                     N, (int)B, (int)H, (int)W, (int)radius, cur_stream()),
              "unsupported radius");
  return out;
}

// writes bf16 taps into channels [0, L*D*D) of an NHWC (B,H,W,Cbuf) buffer (the fused update
// block's correlation input); the caller owns the zero padding of the remaining channels
void corr_lookup_nhwc_(const std::vector<Tensor>& pyr, const Tensor& coords, int64_t radius,
                       const Tensor& out, bool split) {
  check_cuda_f32(coords, "coords");
  TORCH_CHECK(coords.dim() == 4 && coords.size(1) == 2, "coords must be (B,2,H,W)");
  TORCH_CHECK(radius == 3 || radius == 4, "radius must be 3 or 4");
  c10::DeviceGuard g(coords.device());
  const int64_t B = coords.size(0), H = coords.size(2), W = coords.size(3);
  // fp32 or bf16 pyramid (corr_build_bf16 with pyr_bf16)
  const bool pyr_bf16 = !pyr.empty() && pyr[0].scalar_type() == at::kBFloat16;
  std::vector<Tensor> pyr32;
  std::vector<const void*> cp;
  Levels L;
  if (pyr_bf16) {
    TORCH_CHECK(pyr.size() <= 4, "pyramid: 1..4 levels required");
    for (const auto& t : pyr) {
      TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kBFloat16 && t.dim() == 4,
                  "bf16 pyramid levels must be contiguous (B, N, h, w)");
      TORCH_CHECK(t.size(0) * t.size(1) == B * H * W, "pyramid plane count mismatch");
      TORCH_CHECK(t.numel() * 2 < (int64_t(1) << 40), "pyramid level too large");
      cp.push_back(t.data_ptr());
      L.h.push_back((int)t.size(2));
      L.w.push_back((int)t.size(3));
    }
  } else {
    L = levels_of(pyr, B * H * W, "pyramid");
    for (auto* q : L.ptr) cp.push_back(q);
  }
  TORCH_CHECK(L.h[0] == H && L.w[0] == W, "pyramid level 0 must match coords grid");
  const int64_t D = 2 * radius + 1;
  const int levels = (int)pyr.size();
  const bool f16 = out.scalar_type() == at::kHalf;
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && (f16 || out.scalar_type() == at::kBFloat16) &&
                  out.dim() == 4 && out.size(0) == B && out.size(1) == H && out.size(2) == W &&
                  out.size(3) >= (split ? 2 : 1) * levels * D * D,
              "out must be a contiguous bf16 / fp16 (B,H,W,C>=L*D*D) buffer");
  TORCH_CHECK(!(f16 && pyr_bf16), "fp16 taps come from the fp32 pyramid");
  // split fp32 taps: [hi (C/2) | lo (C/2)] bf16 halves from the fp32 pyramid
  TORCH_CHECK(!split || (!f16 && !pyr_bf16 && out.size(3) % 16 == 0), "split taps: bf16 halves, fp32 pyramid");
  const int64_t Cb = split ? out.size(3) / 2 : out.size(3);
  TORCH_CHECK(Cb % 8 == 0, "out channels must be a multiple of 8");
  // LDS-tiled kernel writes whole pixel rows including the zero padding
  TORCH_CHECK(launch_corr_lookup_tile(cp.data(), L.h.data(), L.w.data(), levels,
                                      coords.data_ptr<float>(), reinterpret_cast<uint16_t*>(out.data_ptr()),
                                      (int)Cb, (int)B, (int)H, (int)W, (int)radius, pyr_bf16,
                                      split ? 2 : (f16 ? 1 : 0), cur_stream()),
              "unsupported radius");
}

// per-iteration compact window gradient: (B, N, L, 2r+2, 2r+2) fp32 from a bf16 NHWC tap gradient
Tensor corr_window_grad(const Tensor& coords, const Tensor& dout, int64_t levels, int64_t radius) {
  check_cuda_f32(coords, "coords");
  TORCH_CHECK(coords.dim() == 4 && coords.size(1) == 2, "coords must be (B,2,H,W)");
  TORCH_CHECK(radius == 3 || radius == 4, "radius must be 3 or 4");
  TORCH_CHECK(levels >= 1 && levels <= 4, "levels must be 1..4");
  const int64_t B = coords.size(0), H = coords.size(2), W = coords.size(3);
  const int64_t D = 2 * radius + 1, E = D + 1;
  TORCH_CHECK(dout.is_cuda() && dout.is_contiguous() && dout.scalar_type() == at::kBFloat16 &&
                  dout.dim() == 4 && dout.size(0) == B && dout.size(1) == H && dout.size(2) == W &&
                  dout.size(3) % 8 == 0 && dout.size(3) >= (levels * D * D + 7) / 8 * 8,
              "grad must be a contiguous bf16 (B,H,W,Cbuf) tensor");
  c10::DeviceGuard g(coords.device());
  Tensor wg = at::empty({B, H * W, levels, E, E}, coords.options());
  TORCH_CHECK(launch_corr_window_grad(coords.data_ptr<float>(),
                                      reinterpret_cast<const uint16_t*>(dout.data_ptr<at::BFloat16>()),
                                      (int)dout.size(3), wg.data_ptr<float>(), (int)B, (int)H, (int)W,
                                      (int)levels, (int)radius, cur_stream()),
              "unsupported radius");
  return wg;
}

// sum of all iterations' window gradients -> dcorr (B, N, N) = level-0 gradient * 1/sqrt(C)
Tensor corr_window_reduce(const std::vector<Tensor>& coords, const std::vector<Tensor>& wgs,
                          int64_t H, int64_t W, int64_t levels, int64_t radius, double inv_sqrt_c,
                          bool out_bf16) {
  TORCH_CHECK(!coords.empty() && coords.size() == wgs.size() && coords.size() <= RAFT_MAX_WIN,
              "1..", RAFT_MAX_WIN, " iterations");
  const int64_t B = coords[0].size(0), N = H * W;
  const int64_t E = 2 * radius + 2;
  WinList wl{};
  for (size_t k = 0; k < coords.size(); ++k) {
    check_cuda_f32(coords[k], "coords");
    check_cuda_f32(wgs[k], "window grad");
    TORCH_CHECK(coords[k].dim() == 4 && coords[k].size(0) == B && coords[k].size(1) == 2 &&
                    coords[k].size(2) == H && coords[k].size(3) == W,
                "coords shape");
    TORCH_CHECK(wgs[k].numel() == B * N * levels * E * E, "window grad shape");
    wl.coords[k] = coords[k].data_ptr<float>();
    wl.wg[k] = wgs[k].data_ptr<float>();
  }
  wl.n = (int)coords.size();
  const int lds = corr_window_reduce_lds_bytes((int)H, (int)W, (int)levels);
  TORCH_CHECK(lds <= 64 * 1024, "feature map too large for the LDS plane reduction");
  c10::DeviceGuard g(coords[0].device());
  Tensor out = at::empty({B, N, N}, coords[0].options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  TORCH_CHECK(launch_corr_window_reduce(wl, (int)levels, (int)B, (int)H, (int)W, (int)radius,
                                        (float)inv_sqrt_c, out.data_ptr(), out_bf16 ? 1 : 0, cur_stream()),
              "unsupported radius");
  return out;
}

void corr_lookup_bwd_(const std::vector<Tensor>& gpyr, const Tensor& coords, const Tensor& dout,
                      int64_t radius) {
  check_cuda_f32(coords, "coords");
  check_cuda_f32(dout, "grad_corr");
  TORCH_CHECK(radius == 3 || radius == 4, "radius must be 3 or 4");
  c10::DeviceGuard g(coords.device());
  const int64_t B = coords.size(0), H = coords.size(2), W = coords.size(3);
  Levels L = levels_of(gpyr, B * H * W, "grad pyramid");
  const int64_t D = 2 * radius + 1;
  const int64_t Ct = (int64_t)gpyr.size() * D * D, N = H * W;
  const bool nhwc = dout.dim() == 4 && dout.size(0) == B && dout.size(1) == H && dout.size(2) == W &&
                    dout.size(3) >= Ct;
  const bool nchw = dout.dim() == 4 && dout.size(0) == B && dout.size(1) == Ct && dout.size(2) == H &&
                    dout.size(3) == W;
  TORCH_CHECK(nchw || nhwc, "grad_corr must be (B,L*D*D,H,W) or (B,H,W,C>=L*D*D)");
  const int64_t Cb = nhwc && !nchw ? dout.size(3) : Ct;
  TORCH_CHECK(launch_corr_lookup_bwd(L.ptr.data(), L.h.data(), L.w.data(), (int)gpyr.size(),
                                     coords.data_ptr<float>(), dout.data_ptr<float>(),
                                     nchw ? Ct * N : N * Cb, nchw ? 1 : Cb, nchw ? N : 1, (int)B,
                                     (int)H, (int)W, (int)radius, cur_stream()),
              "unsupported radius");
}

// returns dcorr level-0 as (B, N, N) with the 1/sqrt(C) factor applied
Tensor corr_pyr_grad_reduce(const std::vector<Tensor>& gpyr, double inv_sqrt_c) {
  TORCH_CHECK(!gpyr.empty(), "empty grad pyramid");
  const auto& g0 = gpyr[0];
  c10::DeviceGuard g(g0.device());
  const int64_t B = g0.size(0), N = g0.size(1), H = g0.size(2), W = g0.size(3);
  TORCH_CHECK(N == H * W, "level 0 planes must be H*W");
  Levels L = levels_of(gpyr, B * N, "grad pyramid");
  Tensor out = at::empty({B, N, N}, g0.options());
  launch_corr_pyr_grad_reduce(L.ptr.data(), L.h.data(), L.w.data(), B * N, (int)gpyr.size(),
                              (float)inv_sqrt_c, out.data_ptr<float>(), cur_stream());
  return out;
}

// ------------------------------------------------------------------ on-the-fly correlation
struct Bf16Levels {
  std::vector<const uint16_t*> ptr;
  std::vector<int> h, w;
};

void check_cuda_bf16(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16, got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// fmap2 pyramid (NHWC bf16): level l is (B, floor(h/2^l), floor(w/2^l), C)
Bf16Levels otf_levels(const std::vector<Tensor>& lv, int64_t B, int64_t C, int64_t H, int64_t W) {
  TORCH_CHECK(!lv.empty() && lv.size() <= 4, "fmap2 pyramid: 1..4 levels required");
  Bf16Levels L;
  int64_t h = H, w = W;
  for (const auto& t : lv) {
    check_cuda_bf16(t, "fmap2 level");
    TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == h && t.size(2) == w &&
                    t.size(3) == C,
                "fmap2 level must be (B, h/2^l, w/2^l, C) NHWC");
    TORCH_CHECK(h >= 1 && w >= 1, "feature map too small for the pyramid");
    L.ptr.push_back(reinterpret_cast<const uint16_t*>(t.data_ptr()));
    L.h.push_back((int)h);
    L.w.push_back((int)w);
    h /= 2;
    w /= 2;
  }
  return L;
}

void otf_common_checks(const Tensor& f1, const Tensor& coords, int64_t radius) {
  check_cuda_bf16(f1, "fmap1");
  check_cuda_f32(coords, "coords");
  TORCH_CHECK(f1.dim() == 4, "fmap1 must be (B,H,W,C) NHWC");
  TORCH_CHECK(f1.size(3) == 128 || f1.size(3) == 256, "on-the-fly corr supports C = 128/256");
  TORCH_CHECK(radius == 3 || radius == 4, "radius must be 3 or 4");
  TORCH_CHECK(coords.dim() == 4 && coords.size(0) == f1.size(0) && coords.size(1) == 2 &&
                  coords.size(2) == f1.size(1) && coords.size(3) == f1.size(2),
              "coords must be (B,2,H,W)");
}

// out (B,H,W,S) fp32 or bf16, S >= L*(2r+1)^2; channels past L*(2r+1)^2 are zero-filled
// lo = [] (bf16 operands) or [f1_lo, f2_lo levels...] (split-bf16, fp32-accurate)
void corr_otf_fwd_(const Tensor& f1, const std::vector<Tensor>& f2, const Tensor& coords,
                   int64_t radius, const Tensor& out, const std::vector<Tensor>& lo) {
  otf_common_checks(f1, coords, radius);
  const int64_t B = f1.size(0), H = f1.size(1), W = f1.size(2), C = f1.size(3);
  c10::DeviceGuard g(f1.device());
  Bf16Levels L = otf_levels(f2, B, C, H, W);
  const uint16_t* f1lo = nullptr;
  Bf16Levels LL;
  if (!lo.empty()) {
    TORCH_CHECK(lo.size() == f2.size() + 1, "lo must be [f1_lo, f2_lo levels...]");
    check_cuda_bf16(lo[0], "fmap1 lo");
    TORCH_CHECK(lo[0].sizes() == f1.sizes(), "fmap1 lo shape mismatch");
    f1lo = reinterpret_cast<const uint16_t*>(lo[0].data_ptr());
    LL = otf_levels(std::vector<Tensor>(lo.begin() + 1, lo.end()), B, C, H, W);
  }
  const int64_t D = 2 * radius + 1;
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.dim() == 4 && out.size(0) == B &&
                  out.size(1) == H && out.size(2) == W && out.size(3) >= (int64_t)f2.size() * D * D,
              "out must be contiguous (B,H,W,S) with S >= levels*(2r+1)^2");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16 ||
                  (out.scalar_type() == at::kHalf && f1lo != nullptr),
              "out must be float32 or bfloat16 (float16: the fp32-accurate split forward only)");
  const int omode = out.scalar_type() == at::kHalf ? 2 : (out.scalar_type() == at::kBFloat16 ? 1 : 0);
  TORCH_CHECK(launch_corr_otf_fwd(reinterpret_cast<const uint16_t*>(f1.data_ptr()), L.ptr.data(),
                                  f1lo, f1lo ? LL.ptr.data() : nullptr, L.h.data(), L.w.data(),
                                  (int)f2.size(),
                                  coords.data_ptr<float>(), out.data_ptr(),
                                  omode, (int)out.size(3), (int)B,
                                  (int)C, (int)H, (int)W, (int)radius, cur_stream()),
              "on-the-fly corr supports radius 3/4 with C = 128/256");
}

// deterministic on-the-fly dF2 (default; RAFT_OTF_DF2_ATOMIC=1: float atomics): per-tile slab
// rows sized for a union box of up to 32 x 32 positions at level 0 (~20 x 20 at chairs), 24 x 24
// above; a box past that capacity falls back to atomics for its tile.  The scratch grows with the
// pixel count (~170 KB per query pixel at C = 256) while on-the-fly correlation is what runs when
// the all-pairs pyramid does not fit, so it is bounded: past RAFT_OTF_SLAB_GB (default 8) the
// whole call takes the atomic dF2 path instead of allocating more
struct OtfSlabs {
  std::vector<Tensor> keep;
  std::vector<float*> ptr;
  std::vector<int> cap;
  Tensor boxes;
  bool on = false;
  OtfSlabs(const Bf16Levels& L, int64_t levels, int64_t B, int64_t H, int64_t W, int64_t C,
           const at::TensorOptions& fo) {
    static const bool atomic_df2 = [] {
      const char* e = getenv("RAFT_OTF_DF2_ATOMIC");
      return e && e[0] == '1';
    }();
    const char* eb = getenv("RAFT_OTF_SLAB_GB");   // read per call (tests lower it)
    const double budget = (eb ? atof(eb) : 8.0) * 1e9;
    if (atomic_df2) return;
    const int tiles = otf_tiles((int)B, (int)H, (int)W);
    double bytes = 0.0;
    for (int64_t l = 0; l < levels; ++l) {
      const int plane = L.h[l] * L.w[l];
      cap.push_back(std::min(plane, l == 0 ? 1024 : 576));
      bytes += (double)tiles * cap.back() * C * 4.0;
    }
    if (bytes > budget) {
      cap.clear();
      return;
    }
    on = true;
    for (int64_t l = 0; l < levels; ++l) {
      keep.push_back(at::empty({(int64_t)tiles * cap[l] * C}, fo));
      ptr.push_back(keep.back().data_ptr<float>());
    }
    boxes = at::empty({(int64_t)tiles * 16}, fo.dtype(at::kInt));
  }
  float* const* slab() const { return on ? ptr.data() : nullptr; }
  const int* caps() const { return on ? cap.data() : nullptr; }
  int* box() { return on ? boxes.data_ptr<int>() : nullptr; }
};

void corr_otf_bwd_(const Tensor& f1, const std::vector<Tensor>& f2, const Tensor& coords,
                   const Tensor& dout, const Tensor& df1, const std::vector<Tensor>& df2,
                   int64_t radius, int64_t dslo) {
  otf_common_checks(f1, coords, radius);
  const int64_t B = f1.size(0), H = f1.size(1), W = f1.size(2), C = f1.size(3);
  check_cuda_f32(df1, "grad_fmap1");
  TORCH_CHECK(df1.sizes() == f1.sizes(), "grad_fmap1 must be (B,H,W,C)");
  const int64_t D = 2 * radius + 1;
  TORCH_CHECK(dout.is_cuda() && dout.is_contiguous() && dout.dim() == 4 && dout.size(0) == B &&
                  dout.size(1) == H && dout.size(2) == W &&
                  dout.size(3) >= (int64_t)f2.size() * D * D,
              "grad_corr must be contiguous (B,H,W,S) with S >= levels*(2r+1)^2");
  TORCH_CHECK(dout.scalar_type() == at::kFloat || dout.scalar_type() == at::kBFloat16,
              "grad_corr must be float32 or bfloat16");
  TORCH_CHECK(f2.size() == df2.size(), "level count mismatch");
  c10::DeviceGuard g(f1.device());
  Bf16Levels L = otf_levels(f2, B, C, H, W);
  std::vector<float*> gp;
  for (size_t l = 0; l < df2.size(); ++l) {
    check_cuda_f32(df2[l], "grad fmap2 level");
    TORCH_CHECK(df2[l].sizes() == f2[l].sizes(), "grad fmap2 level shape mismatch");
    gp.push_back(df2[l].data_ptr<float>());
  }
  OtfSlabs sl(L, (int64_t)f2.size(), B, H, W, C, df1.options());
  TORCH_CHECK(launch_corr_otf_bwd(reinterpret_cast<const uint16_t*>(f1.data_ptr()), L.ptr.data(),
                                  L.h.data(), L.w.data(), (int)f2.size(),
                                  coords.data_ptr<float>(), dout.data_ptr(),
                                  dout.scalar_type() == at::kBFloat16, (int)dout.size(3),
                                  df1.data_ptr<float>(), gp.data(), (int)B, (int)C, (int)H, (int)W,
                                  (int)radius, sl.slab(), sl.caps(), sl.box(), (int)dslo,
                                  cur_stream()),
              "on-the-fly corr supports radius 3/4 with C = 128/256");
}

// every iteration's gradient at once: coords[k] (B,2,H,W) and douts[k] (B,H,W,cbuf) bf16, the
// gradient of iteration k's NHWC lookup output (taps in channels [0, L*(2r+1)^2))
void corr_otf_window_bwd_(const Tensor& f1, const std::vector<Tensor>& f2,
                          const std::vector<Tensor>& coords, const std::vector<Tensor>& douts,
                          const Tensor& df1, const std::vector<Tensor>& df2, int64_t radius) {
  TORCH_CHECK(!coords.empty() && coords.size() == douts.size() && coords.size() <= RAFT_MAX_WIN,
              "1..", RAFT_MAX_WIN, " iterations");
  otf_common_checks(f1, coords[0], radius);
  const int64_t B = f1.size(0), H = f1.size(1), W = f1.size(2), C = f1.size(3);
  const int64_t levels = (int64_t)f2.size(), D = 2 * radius + 1;
  check_cuda_f32(df1, "grad_fmap1");
  TORCH_CHECK(df1.sizes() == f1.sizes(), "grad_fmap1 must be (B,H,W,C)");
  TORCH_CHECK(f2.size() == df2.size(), "level count mismatch");
  WinList wl{};
  const int64_t cbuf = douts[0].dim() == 4 ? douts[0].size(3) : 0;
  for (size_t k = 0; k < coords.size(); ++k) {
    check_cuda_f32(coords[k], "coords");
    TORCH_CHECK(coords[k].sizes() == coords[0].sizes(), "coords shape");
    TORCH_CHECK(douts[k].is_cuda() && douts[k].is_contiguous() && douts[k].scalar_type() == at::kBFloat16 &&
                    douts[k].dim() == 4 && douts[k].size(0) == B && douts[k].size(1) == H &&
                    douts[k].size(2) == W && douts[k].size(3) == cbuf,
                "tap gradients must be contiguous bf16 (B,H,W,Cbuf) tensors of one shape");
    wl.coords[k] = coords[k].data_ptr<float>();
    wl.dout[k] = reinterpret_cast<const uint16_t*>(douts[k].data_ptr<at::BFloat16>());
  }
  // the kernel stages 16-B pieces of the 8-aligned span of every level's taps
  TORCH_CHECK(cbuf % 8 == 0 && cbuf >= (levels * D * D + 7) / 8 * 8, "tap gradient Cbuf too small");
  wl.cbuf = (int)cbuf;
  wl.n = (int)coords.size();
  c10::DeviceGuard g(f1.device());
  Bf16Levels L = otf_levels(f2, B, C, H, W);
  std::vector<float*> gp;
  for (size_t l = 0; l < df2.size(); ++l) {
    check_cuda_f32(df2[l], "grad fmap2 level");
    TORCH_CHECK(df2[l].sizes() == f2[l].sizes(), "grad fmap2 level shape mismatch");
    gp.push_back(df2[l].data_ptr<float>());
  }
  OtfSlabs sl(L, levels, B, H, W, C, df1.options());
  // the coarse levels' dF1 part (two workgroups per query tile; summed into df1 in fixed order)
  Tensor df1b;
  if (levels >= 2) df1b = at::empty_like(df1, at::MemoryFormat::Contiguous);
  TORCH_CHECK(launch_corr_otf_window_bwd(reinterpret_cast<const uint16_t*>(f1.data_ptr()),
                                         L.ptr.data(), L.h.data(), L.w.data(), (int)levels, wl,
                                         df1.data_ptr<float>(), gp.data(), (int)B, (int)C, (int)H,
                                         (int)W, (int)radius, sl.slab(), sl.caps(), sl.box(),
                                         df1b.defined() ? df1b.data_ptr<float>() : nullptr,
                                         cur_stream()),
              "on-the-fly corr supports radius 3/4 with C = 128/256");
}

// ------------------------------------------------------------------ convex upsample
// 0 fp32, 1 bf16, 2 fp16 (fp16 masks: the NHWC fused-path kernels only)
int mask_kind(const Tensor& m) {
  TORCH_CHECK(m.scalar_type() == at::kFloat || m.scalar_type() == at::kBFloat16 ||
                  m.scalar_type() == at::kHalf,
              "mask must be float32, bfloat16 or float16");
  return m.scalar_type() == at::kBFloat16 ? 1 : (m.scalar_type() == at::kHalf ? 2 : 0);
}

// the NHWC vector kernels move the mask / dmask in 8-B and flow / dout / out in 16-B accesses:
// a contiguous view with an odd storage offset (a narrowed tensor) takes the scalar kernels
bool aligned16(const Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }

// mask is (B,576,H,W) contiguous (nhwc=false) or (B,H,W,576) contiguous (nhwc=true)
void check_mask(const Tensor& mask, int64_t B, int64_t H, int64_t W, bool nhwc) {
  TORCH_CHECK(mask.is_cuda() && mask.is_contiguous(), "mask must be a contiguous GPU tensor");
  const bool ok = nhwc ? (mask.dim() == 4 && mask.size(0) == B && mask.size(1) == H &&
                          mask.size(2) == W && mask.size(3) == 576)
                       : (mask.dim() == 4 && mask.size(0) == B && mask.size(1) == 576 &&
                          mask.size(2) == H && mask.size(3) == W);
  TORCH_CHECK(ok, nhwc ? "mask must be (B,H,W,576)" : "mask must be (B,576,H,W)");
}

Tensor convex_up_fwd(const Tensor& flow, const Tensor& mask, bool nhwc) {
  check_cuda_f32(flow, "flow");
  TORCH_CHECK(flow.dim() == 4 && flow.size(1) == 2, "flow must be (B,2,H,W)");
  const int64_t B = flow.size(0), H = flow.size(2), W = flow.size(3);
  check_mask(mask, B, H, W, nhwc);
  c10::DeviceGuard g(flow.device());
  Tensor out = at::empty({B, 2, 8 * H, 8 * W}, flow.options());
  const int64_t HW = H * W;
  if (nhwc && mask.is_contiguous() && aligned16(flow) && aligned16(mask) && aligned16(out)) {
    launch_convex_up_nhwc_fwd(flow.data_ptr<float>(), mask.data_ptr(), mask_kind(mask),
                              out.data_ptr<float>(), (int)B, (int)H, (int)W, cur_stream());
    return out;
  }
  TORCH_CHECK(mask_kind(mask) != 2, "fp16 masks need the aligned NHWC layout");
  launch_convex_up_fwd(flow.data_ptr<float>(), mask.data_ptr(), mask_kind(mask), 576 * HW,
                       nhwc ? 1 : HW, nhwc ? 576 : 1, out.data_ptr<float>(), (int)B, (int)H,
                       (int)W, cur_stream());
  return out;
}

std::vector<Tensor> convex_up_bwd(const Tensor& flow, const Tensor& mask, const Tensor& dout,
                                  bool nhwc) {
  check_cuda_f32(flow, "flow");
  check_cuda_f32(dout, "grad_out");
  const int64_t B = flow.size(0), H = flow.size(2), W = flow.size(3);
  check_mask(mask, B, H, W, nhwc);
  TORCH_CHECK(dout.dim() == 4 && dout.size(0) == B && dout.size(1) == 2 && dout.size(2) == 8 * H &&
                  dout.size(3) == 8 * W,
              "grad_out must be (B,2,8H,8W)");
  c10::DeviceGuard g(flow.device());
  Tensor dmask = at::empty_like(mask);
  Tensor dflow = at::empty_like(flow);
  Tensor wbuf = at::empty({B, 18, H, W}, flow.options());
  const int64_t HW = H * W;
  if (nhwc && mask.is_contiguous() && dmask.is_contiguous() && aligned16(flow) && aligned16(mask) &&
      aligned16(dout) && aligned16(dmask) && aligned16(dflow)) {
    launch_convex_up_nhwc_bwd(flow.data_ptr<float>(), mask.data_ptr(), mask_kind(mask),
                              dout.data_ptr<float>(), dmask.data_ptr(), wbuf.data_ptr<float>(),
                              dflow.data_ptr<float>(), (int)B, (int)H, (int)W, cur_stream());
    return {dflow, dmask};
  }
  TORCH_CHECK(mask_kind(mask) != 2, "fp16 masks need the aligned NHWC layout");
  launch_convex_up_bwd(flow.data_ptr<float>(), mask.data_ptr(), mask_kind(mask), 576 * HW,
                       nhwc ? 1 : HW, nhwc ? 576 : 1, dout.data_ptr<float>(), dmask.data_ptr(),
                       wbuf.data_ptr<float>(), dflow.data_ptr<float>(), (int)B, (int)H, (int)W,
                       cur_stream());
  return {dflow, dmask};
}

// ------------------------------------------------------------------ sequence loss
void check_preds(const std::vector<Tensor>& preds, const Tensor& gt) {
  TORCH_CHECK(!preds.empty() && preds.size() <= RAFT_MAX_PREDS, "1..", RAFT_MAX_PREDS,
              " predictions supported");
  check_cuda_f32(gt, "flow_gt");
  TORCH_CHECK(gt.dim() == 4 && gt.size(1) == 2, "flow_gt must be (B,2,H,W)");
  for (const auto& p : preds) {
    check_cuda_f32(p, "flow_pred");
    TORCH_CHECK(p.sizes() == gt.sizes(), "prediction / ground-truth shape mismatch");
  }
}

Tensor seq_loss_fwd(const std::vector<Tensor>& preds, const Tensor& gt, const Tensor& valid,
                    double gamma, double max_flow) {
  check_preds(preds, gt);
  check_cuda_f32(valid, "valid");
  const int64_t B = gt.size(0), HW = gt.size(2) * gt.size(3);
  TORCH_CHECK(valid.numel() == B * HW, "valid must be (B,H,W)");
  c10::DeviceGuard g(gt.device());
  PredPtrs P;
  for (size_t i = 0; i < preds.size(); ++i) P.p[i] = preds[i].data_ptr<float>();
  Tensor partial = at::empty({seq_loss_partial_count()}, gt.options());
  Tensor out = at::empty({6}, gt.options());
  launch_seq_loss_fwd(P, (int)preds.size(), gt.data_ptr<float>(), valid.data_ptr<float>(),
                      (float)gamma, (float)max_flow, (int)B, HW, partial.data_ptr<float>(),
                      out.data_ptr<float>(), cur_stream());
  return out;
}

std::vector<Tensor> seq_loss_bwd(const std::vector<Tensor>& preds, const Tensor& gt,
                                 const Tensor& valid, const Tensor& dloss, double gamma,
                                 double max_flow) {
  check_preds(preds, gt);
  check_cuda_f32(valid, "valid");
  check_cuda_f32(dloss, "grad_loss");
  TORCH_CHECK(dloss.numel() >= 1, "grad_loss must hold one value");
  const int64_t B = gt.size(0), HW = gt.size(2) * gt.size(3);
  TORCH_CHECK(valid.numel() == B * HW, "valid must be (B,H,W)");
  c10::DeviceGuard g(gt.device());
  PredPtrs P;
  PredPtrsMut G;
  std::vector<Tensor> grads;
  for (size_t i = 0; i < preds.size(); ++i) {
    P.p[i] = preds[i].data_ptr<float>();
    grads.push_back(at::empty_like(preds[i]));
    G.p[i] = grads.back().data_ptr<float>();
  }
  launch_seq_loss_bwd(P, G, (int)preds.size(), gt.data_ptr<float>(), valid.data_ptr<float>(),
                      dloss.data_ptr<float>(), (float)gamma, (float)max_flow, (int)B, HW,
                      cur_stream());
  return grads;
}

// ------------------------------------------------------------------ warping sampler
void check_warp(const Tensor& img, const Tensor& flow) {
  check_cuda_f32(img, "image");
  check_cuda_f32(flow, "flow");
  TORCH_CHECK(img.dim() == 4 && flow.dim() == 4 && flow.size(1) == 2 && img.size(0) == flow.size(0) &&
                  img.size(2) == flow.size(2) && img.size(3) == flow.size(3),
              "image (B,C,H,W) and flow (B,2,H,W) must match");
}

Tensor warp_fwd(const Tensor& img, const Tensor& flow, double sx, double bx, double sy, double by) {
  check_warp(img, flow);
  c10::DeviceGuard g(img.device());
  Tensor out = at::empty_like(img);
  launch_warp_fwd(img.data_ptr<float>(), flow.data_ptr<float>(), out.data_ptr<float>(),
                  (int)img.size(0), (int)img.size(1), (int)img.size(2), (int)img.size(3), (float)sx,
                  (float)bx, (float)sy, (float)by, cur_stream());
  return out;
}

std::vector<Tensor> warp_bwd(const Tensor& img, const Tensor& flow, const Tensor& dout, double sx,
                             double bx, double sy, double by) {
  check_warp(img, flow);
  check_cuda_f32(dout, "grad_out");
  TORCH_CHECK(dout.sizes() == img.sizes(), "grad_out shape mismatch");
  c10::DeviceGuard g(img.device());
  Tensor dimg = at::zeros_like(img);
  Tensor dflow = at::empty_like(flow);
  launch_warp_bwd(img.data_ptr<float>(), flow.data_ptr<float>(), dout.data_ptr<float>(),
                  dimg.data_ptr<float>(), dflow.data_ptr<float>(), (int)img.size(0),
                  (int)img.size(1), (int)img.size(2), (int)img.size(3), (float)sx, (float)bx,
                  (float)sy, (float)by, cur_stream());
  return {dimg, dflow};
}

// ------------------------------------------------------------------ implicit-GEMM convolution
// All activations are NHWC bf16 tensors of shape (B, H, W, C_buffer); a "segment" is a channel
// slice [off, off + cnt) of such a buffer.  Geometry is validated here so the kernel's pointer
// arithmetic can never leave an allocation.
void check_nhwc(const Tensor& t, int64_t B, int64_t H, int64_t W, const char* name, at::ScalarType st) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
  TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == H && t.size(2) == W, name,
              " must be (B,H,W,C) matching the conv geometry");
}

// 16-bit operand type of the MFMA kernels: bf16 (default) or fp16 (fp16 autocast)
at::ScalarType op16(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf,
              "16-bit operands must be bfloat16 or float16, got ", t.scalar_type());
  return t.scalar_type();
}
const uint16_t* u16(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* u16m(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

void conv_fwd_(const std::vector<Tensor>& ins, const std::vector<int64_t>& in_off,
               const std::vector<int64_t>& in_cnt, const Tensor& wpk,
               const c10::optional<Tensor>& bias, int64_t kh, int64_t kw, int64_t ph, int64_t pw,
               int64_t cout, int64_t cin_small, int64_t epi, int64_t bn, double scale,
               int64_t split, const std::vector<Tensor>& outs, const std::vector<int64_t>& out_off,
               const std::vector<Tensor>& aux, const std::vector<int64_t>& aux_off) {
  TORCH_CHECK(!ins.empty() && ins.size() <= 3, "1..3 input segments");
  TORCH_CHECK(in_off.size() == ins.size() && in_cnt.size() == ins.size(), "segment spec mismatch");
  TORCH_CHECK(bn == 128 || bn == 64 || bn == 32, "bn must be 128/64/32");
  const int64_t B = ins[0].size(0), H = ins[0].size(1), W = ins[0].size(2);
  c10::DeviceGuard g(ins[0].device());
  ConvFwdArgs a{};
  const at::ScalarType st = op16(ins[0]);
  TORCH_CHECK(!epi_f16((int)epi), "pass the epilogue kind; fp16 follows the operand dtype");
  // split fp32 (EPI_SPL): every 16-bit tensor holds [hi | lo] halves; segments, output and aux
  // slices name hi-half channels, the kernels find the lo half at + size(3) / 2
  const bool spl = epi_spl((int)epi);
  epi = epi_kind((int)epi);
  TORCH_CHECK(!spl || (st == at::kBFloat16 && cin_small == 0), "split fp32: bf16 pairs, no small-Cin path");
  auto half = [&](const Tensor& t) -> int64_t {
    if (!spl) return t.size(3);
    TORCH_CHECK(t.size(3) % 16 == 0, "split fp32 tensors hold two 8-aligned halves");
    return t.size(3) / 2;
  };
  a.nseg = (int)ins.size();
  int64_t cin_pad = 0;
  for (size_t s = 0; s < ins.size(); ++s) {
    check_nhwc(ins[s], B, H, W, "conv input", st);
    // a segment may run past the tensor's last channel (a 96-channel tensor in a 128-channel K
    // slot): the kernels read the channels that are not there as zeros
    const int64_t present = std::min<int64_t>(in_cnt[s], half(ins[s]) - in_off[s]);
    TORCH_CHECK(in_off[s] >= 0 && present > 0 && present % 8 == 0 &&
                    (present == in_cnt[s] || cin_small == 0),
                "segment out of range");
    TORCH_CHECK(in_off[s] % 8 == 0 && ins[s].size(3) % 8 == 0, "segments must be 16-byte aligned");
    if (cin_small == 0) TORCH_CHECK(in_cnt[s] % 64 == 0, "segment channels must be a multiple of 64");
    TORCH_CHECK(ins[s].numel() * 2 < (int64_t(1) << 31), "conv input exceeds the 2 GiB buffer-descriptor range");
    a.seg[s].ptr = u16(ins[s]) + in_off[s];
    a.seg[s].stride = (int)ins[s].size(3);
    a.seg[s].cnt = (int)in_cnt[s];
    a.seg[s].real = (int)present;
    cin_pad += in_cnt[s];
  }
  if (spl) cin_pad *= 3;  // K thirds [hi | lo | hi]
  a.spl = spl ? 1 : 0;
  a.cin_pad = (int)cin_pad;
  a.cin_small = (int)cin_small;
  if (cin_small) TORCH_CHECK(ins.size() == 1 && cin_small <= in_cnt[0], "small-Cin path takes one segment");
  a.B = (int)B; a.H = (int)H; a.W = (int)W;
  a.KH = (int)kh; a.KW = (int)kw; a.PH = (int)ph; a.PW = (int)pw;
  TORCH_CHECK(wpk.is_cuda() && wpk.is_contiguous() && wpk.scalar_type() == st && wpk.dim() == 2,
              "packed weight must be a contiguous (Npad, Kpad) tensor of the operand dtype");
  const int64_t kneed = cin_small ? ((kh * kw * cin_small + 63) / 64) * 64 : kh * kw * cin_pad;
  TORCH_CHECK(wpk.size(1) == kneed, "packed weight K mismatch: ", wpk.size(1), " vs ", kneed);
  // rows past cout are never read (range-checked descriptors in every kernel)
  TORCH_CHECK(wpk.size(0) >= cout, "packed weight has too few rows");
  a.wpk = u16(wpk);
  a.kpad = (int)wpk.size(1);
  if (bias.has_value() && bias->defined() && bias->dim() == 4) {
    // per-pixel bias map (B,H,W,>=cout) fp32 or bf16: the precomputed context part of a ConvGRU conv
    TORCH_CHECK(epi == EPI_GRU_ZR || epi == EPI_GRU_Q, "a per-pixel bias map needs a GRU epilogue");
    const bool bm16 = bias->scalar_type() != at::kFloat;
    check_nhwc(*bias, B, H, W, "bias map", bm16 ? st : at::kFloat);
    TORCH_CHECK(bias->size(3) >= cout, "bias map has too few channels");
    TORCH_CHECK(bias->numel() * bias->element_size() < (int64_t(1) << 31),
                "bias map exceeds the 2 GiB buffer-descriptor range");
    a.bmap = reinterpret_cast<const float*>(bias->data_ptr());
    a.bmap_stride = (int)bias->size(3);
    a.bmap_bf16 = bm16 ? 1 : 0;
  } else if (bias.has_value() && bias->defined()) {
    check_cuda_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() >= cout, "bias too short");
    a.bias = bias->data_ptr<float>();
  }
  const int ef16 = st == at::kHalf ? EPI_F16 : 0;
  TORCH_CHECK(!ef16 || cin_small == 0, "fp16 operands: no small-Cin path");
  a.cout = (int)cout;
  a.scale = (float)scale;
  a.split = (int)split;
  // the epilogue picks the z / r half per 32-column MFMA tile
  TORCH_CHECK(epi != EPI_GRU_ZR || (split % 32 == 0 && split > 0 && split < cout),
              "GRU z|r split must be a multiple of 32");
  TORCH_CHECK(epi != EPI_DGRAD, "use conv_dgrad_ for the dgrad epilogue");
  const bool f32out = (epi == EPI_F32 || epi == EPI_ACC_F32 || epi == EPI_F32_NCHW);
  const int64_t need_out = (epi == EPI_GRU_ZR) ? 3 : (epi == EPI_GRU_Q ? 2 : 1);
  TORCH_CHECK((int64_t)outs.size() == need_out && out_off.size() == outs.size(), "wrong output count");
  if (epi == EPI_F32_NCHW) {
    const Tensor& o = outs[0];
    TORCH_CHECK(o.is_cuda() && o.is_contiguous() && o.scalar_type() == at::kFloat && o.dim() == 4 &&
                    o.size(0) == B && o.size(1) == cout && o.size(2) == H && o.size(3) == W &&
                    out_off[0] == 0,
                "NCHW output must be a contiguous fp32 (B,cout,H,W) tensor");
    a.out0 = o.data_ptr<float>();
    a.out0_stride = 0;
    TORCH_CHECK(aux.empty(), "no aux for the NCHW epilogue");
    TORCH_CHECK(launch_conv_fwd(a, (int)epi | ef16 | (spl ? EPI_SPL : 0), (int)bn, cin_small != 0, cur_stream()),
                "bad epilogue");
    return;
  }
  const int64_t out_ch[3] = {epi == EPI_GRU_ZR ? split : cout, epi == EPI_GRU_ZR ? cout - split : cout,
                             cout - split};
  void** optr[3] = {&a.out0, &a.out1, &a.out2};
  int* ostr[3] = {&a.out0_stride, &a.out1_stride, &a.out2_stride};
  for (size_t o = 0; o < outs.size(); ++o) {
    check_nhwc(outs[o], B, H, W, "conv output", f32out ? at::kFloat : st);
    TORCH_CHECK(outs[o].numel() * outs[o].element_size() < (int64_t(1) << 31),
                "conv output exceeds the 2 GiB buffer-descriptor range");
    TORCH_CHECK(out_off[o] >= 0 && out_off[o] + out_ch[o] <= (f32out ? outs[o].size(3) : half(outs[o])),
                "output slice out of range");
    *optr[o] = f32out ? (void*)(outs[o].data_ptr<float>() + out_off[o])
                      : (void*)(u16m(outs[o]) + out_off[o]);
    *ostr[o] = (int)outs[o].size(3);
  }
  const int64_t need_aux = (epi == EPI_GRU_ZR) ? 1 : (epi == EPI_GRU_Q ? 2 : 0);
  TORCH_CHECK((int64_t)aux.size() == need_aux && aux_off.size() == aux.size(), "wrong aux count");
  const uint16_t** aptr[2] = {&a.aux0, &a.aux1};
  int* astr[2] = {&a.aux0_stride, &a.aux1_stride};
  for (size_t o = 0; o < aux.size(); ++o) {
    check_nhwc(aux[o], B, H, W, "conv aux", st);
    TORCH_CHECK(aux[o].numel() * 2 < (int64_t(1) << 31), "conv aux exceeds the 2 GiB buffer-descriptor range");
    const int64_t ch = (epi == EPI_GRU_ZR) ? cout - split : cout;
    TORCH_CHECK(aux_off[o] >= 0 && aux_off[o] + ch <= half(aux[o]), "aux slice out of range");
    *aptr[o] = u16(aux[o]) + aux_off[o];
    *astr[o] = (int)aux[o].size(3);
  }
  TORCH_CHECK(launch_conv_fwd(a, (int)epi | ef16 | (spl ? EPI_SPL : 0), (int)bn, cin_small != 0, cur_stream()),
              "bad epilogue");
}

std::vector<int64_t> conv_tune_table() {
  std::vector<int> buf(13 * 512);
  const int n = conv_tuned_table(buf.data(), 512);
  return std::vector<int64_t>(buf.begin(), buf.begin() + 13 * n);
}

// dw (cout, kpad) fp32 += sum_p g[p][:cout] (x) im2col(ins)[p][:]; db (cout) fp32 += colsum(g)
void conv_wgrad_(const Tensor& g, int64_t g_off, const std::vector<Tensor>& ins,
                 const std::vector<int64_t>& in_off, const std::vector<int64_t>& in_cnt,
                 int64_t kh, int64_t kw, int64_t ph, int64_t pw, int64_t cout, int64_t cin_small,
                 const Tensor& dw, const c10::optional<Tensor>& db, int64_t pix_per_split) {
  TORCH_CHECK(!ins.empty() && ins.size() <= 3, "1..3 input segments");
  const int64_t B = g.size(0), H = g.size(1), W = g.size(2);
  check_nhwc(g, B, H, W, "grad", at::kBFloat16);
  // the kernel reads G in whole 8-channel chunks: the slice rounded up to 8 must lie in the row
  TORCH_CHECK(g_off >= 0 && g_off % 8 == 0 && g_off + (cout + 7) / 8 * 8 <= g.size(3),
              "grad slice out of range (cout rounded up to 8 channels must fit the row)");
  TORCH_CHECK(g.numel() * 2 < (int64_t(1) << 31), "grad exceeds the 2 GiB buffer-descriptor range");
  c10::DeviceGuard gd(g.device());
  ConvWgradArgs a{};
  a.g = reinterpret_cast<const uint16_t*>(g.data_ptr<at::BFloat16>()) + g_off;
  a.g_stride = (int)g.size(3);
  a.nseg = (int)ins.size();
  int64_t cin_pad = 0;
  for (size_t s = 0; s < ins.size(); ++s) {
    check_nhwc(ins[s], B, H, W, "wgrad input", at::kBFloat16);
    TORCH_CHECK(in_off[s] >= 0 && in_off[s] + in_cnt[s] <= ins[s].size(3), "segment out of range");
    TORCH_CHECK(in_off[s] % 8 == 0 && ins[s].size(3) % 8 == 0, "segments must be 16-byte aligned");
    if (cin_small == 0) TORCH_CHECK(in_cnt[s] % 8 == 0, "segment channels must be a multiple of 8");
    TORCH_CHECK(ins[s].numel() * 2 < (int64_t(1) << 31), "wgrad input exceeds the 2 GiB buffer-descriptor range");
    TORCH_CHECK(ins[s].numel() * 2 < (int64_t(1) << 31), "conv input exceeds the 2 GiB buffer-descriptor range");
    a.seg[s].ptr = reinterpret_cast<const uint16_t*>(ins[s].data_ptr<at::BFloat16>()) + in_off[s];
    a.seg[s].stride = (int)ins[s].size(3);
    a.seg[s].cnt = (int)in_cnt[s];
    a.seg[s].real = (int)in_cnt[s];
    cin_pad += in_cnt[s];
  }
  a.cin_pad = (int)cin_pad;
  a.cin_small = (int)cin_small;
  a.B = (int)B; a.H = (int)H; a.W = (int)W;
  a.KH = (int)kh; a.KW = (int)kw; a.PH = (int)ph; a.PW = (int)pw;
  a.cout = (int)cout;
  check_cuda_f32(dw, "grad_weight");
  const int64_t kpad = cin_small ? ((kh * kw * cin_small + 63) / 64) * 64 : kh * kw * cin_pad;
  TORCH_CHECK(dw.dim() == 2 && dw.size(0) == cout && dw.size(1) == kpad, "grad_weight must be (cout, kpad)");
  a.dw = dw.data_ptr<float>();
  a.kpad = (int)kpad;
  a.pix_per_split = (int)std::max<int64_t>(64, (pix_per_split + 63) / 64 * 64);
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    check_cuda_f32(*db, "grad_bias");
    TORCH_CHECK(db->numel() == cout, "grad_bias size");
    dbp = db->data_ptr<float>();
  }
  launch_conv_wgrad(a, cout > 64 ? 128 : 64, cin_small != 0, dbp, cur_stream());
}

// Weight / bias gradient summed over several (grad, input) items of the same conv geometry -- the
// GRU iterations of one step (shared weights): one launch, split-K over (item, pixel range).
// gs[i] is item i's bf16 NHWC gradient; ins[i * nseg + s] its s-th input segment buffer.
void conv_wgrad_multi_(const std::vector<Tensor>& gs, int64_t g_off, const std::vector<Tensor>& ins,
                       const std::vector<int64_t>& in_off, const std::vector<int64_t>& in_cnt,
                       int64_t kh, int64_t kw, int64_t ph, int64_t pw, int64_t cout,
                       const Tensor& dw, const c10::optional<Tensor>& db, int64_t pix_per_split) {
  const int64_t n = (int64_t)gs.size();
  const int64_t nseg = (int64_t)in_off.size();
  TORCH_CHECK(n >= 1 && n <= RAFT_WG_MAX_ITEMS, "1..", RAFT_WG_MAX_ITEMS, " items");
  TORCH_CHECK(nseg >= 1 && nseg <= 3 && (int64_t)in_cnt.size() == nseg, "1..3 input segments");
  TORCH_CHECK((int64_t)ins.size() == n * nseg, "ins must hold items x segments tensors");
  const Tensor& g0 = gs[0];
  const int64_t B = g0.size(0), H = g0.size(1), W = g0.size(2);
  c10::DeviceGuard gd(g0.device());
  ConvWgradArgs a{};
  WgradItems it{};
  it.n = (int)n;
  a.g_stride = (int)g0.size(3);
  a.nseg = (int)nseg;
  int64_t cin_pad = 0;
  for (int64_t s = 0; s < nseg; ++s) {
    TORCH_CHECK(in_cnt[s] % 128 == 0 && in_off[s] % 8 == 0,
                "multi-item wgrad: segments must be multiples of the 128-wide K tile");
    a.seg[s].stride = (int)ins[s].size(3);
    a.seg[s].cnt = (int)in_cnt[s];
    a.seg[s].real = (int)in_cnt[s];
    cin_pad += in_cnt[s];
  }
  for (int64_t i = 0; i < n; ++i) {
    const Tensor& g = gs[i];
    check_nhwc(g, B, H, W, "grad", at::kBFloat16);
    TORCH_CHECK(g.size(3) == a.g_stride, "all items' grads must share a layout");
    TORCH_CHECK(g_off >= 0 && g_off % 8 == 0 && g_off + (cout + 7) / 8 * 8 <= g.size(3),
                "grad slice out of range (cout rounded up to 8 channels must fit the row)");
    TORCH_CHECK(g.numel() * 2 < (int64_t(1) << 31), "grad exceeds the 2 GiB buffer-descriptor range");
    it.g[i] = reinterpret_cast<const uint16_t*>(g.data_ptr<at::BFloat16>()) + g_off;
    for (int64_t s = 0; s < nseg; ++s) {
      const Tensor& x = ins[i * nseg + s];
      check_nhwc(x, B, H, W, "wgrad input", at::kBFloat16);
      TORCH_CHECK(x.size(3) == a.seg[s].stride, "all items' inputs must share a layout");
      TORCH_CHECK(in_off[s] + in_cnt[s] <= x.size(3), "segment out of range");
      TORCH_CHECK(x.numel() * 2 < (int64_t(1) << 31), "wgrad input exceeds the 2 GiB buffer-descriptor range");
      it.seg[i][s] = reinterpret_cast<const uint16_t*>(x.data_ptr<at::BFloat16>()) + in_off[s];
    }
  }
  a.cin_pad = (int)cin_pad;
  a.B = (int)B; a.H = (int)H; a.W = (int)W;
  a.KH = (int)kh; a.KW = (int)kw; a.PH = (int)ph; a.PW = (int)pw;
  a.cout = (int)cout;
  check_cuda_f32(dw, "grad_weight");
  const int64_t kpad = kh * kw * cin_pad;
  TORCH_CHECK(kpad % 128 == 0, "multi-item wgrad needs packed K a multiple of 128");
  TORCH_CHECK(dw.dim() == 2 && dw.size(0) == cout && dw.size(1) == kpad, "grad_weight must be (cout, kpad)");
  a.dw = dw.data_ptr<float>();
  a.kpad = (int)kpad;
  const int64_t P = B * H * W;
  a.pix_per_split = (int)std::max<int64_t>(64, (pix_per_split + 63) / 64 * 64);
  a.splits_per_item = (int)((P + a.pix_per_split - 1) / a.pix_per_split);
  TORCH_CHECK(W >= 2 && H * W >= 128, "multi-item wgrad needs W >= 2 and H*W >= 128");
  a.w_magic = (uint32_t)(((uint64_t(1) << 32) + (uint64_t)W - 1) / (uint64_t)W);
  TORCH_CHECK((int64_t)n * a.splits_per_item < 65536, "too many splits");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    check_cuda_f32(*db, "grad_bias");
    TORCH_CHECK(db->numel() == cout, "grad_bias size");
    dbp = db->data_ptr<float>();
  }
  TORCH_CHECK(launch_conv_wgrad_multi(a, it, cout > 64 ? 128 : 64, dbp, cur_stream()), "wgrad launch");
}

// Tap-fused multi-item weight gradient (conv_wgrad_taps.hip): same contract as conv_wgrad_multi_
// (dw / db accumulated), segments only need to be multiples of 64 channels.
void conv_wgrad_taps_(const std::vector<Tensor>& gs, int64_t g_off, const std::vector<Tensor>& ins,
                      const std::vector<int64_t>& in_off, const std::vector<int64_t>& in_cnt,
                      int64_t kh, int64_t kw, int64_t ph, int64_t pw, int64_t cout,
                      const Tensor& dw, const c10::optional<Tensor>& db, int64_t splits,
                      bool split) {
  const int64_t n0 = (int64_t)gs.size();
  // split fp32: g and the inputs are [hi | lo] pairs; dW = sum g_hi x_hi + g_lo x_hi + g_hi x_lo
  // as three kernel items per item (the bias sum takes the first two: g_hi + g_lo)
  const int64_t n = split ? 3 * n0 : n0;
  const int64_t nseg = (int64_t)in_off.size();
  TORCH_CHECK(n0 >= 1 && n <= RAFT_WG_MAX_ITEMS, "1..", split ? RAFT_WG_MAX_ITEMS / 3 : RAFT_WG_MAX_ITEMS,
              " items");
  TORCH_CHECK(nseg >= 1 && nseg <= 3 && (int64_t)in_cnt.size() == nseg, "1..3 input segments");
  TORCH_CHECK((int64_t)ins.size() == n0 * nseg, "ins must hold items x segments tensors");
  TORCH_CHECK(!split || op16(gs.at(0)) == at::kBFloat16, "split fp32: bf16 pairs");
  TORCH_CHECK((kh == 1 && kw == 1) || (kh == 1 && kw == 5) || (kh == 5 && kw == 1) ||
                  (kh == 3 && kw == 3),
              "tap-fused wgrad supports 1x1, 1x5, 5x1 and 3x3 kernels");
  const Tensor& g0 = gs[0];
  const int64_t B = g0.size(0), H = g0.size(1), W = g0.size(2);
  c10::DeviceGuard gd(g0.device());
  ConvWgradArgs a{};
  const at::ScalarType st = op16(gs.at(0));
  a.f16 = st == at::kHalf ? 1 : 0;
  WgradItems it{};
  WgradTapArgs ta{};
  it.n = (int)n;
  a.g_stride = (int)g0.size(3);
  a.nseg = (int)nseg;
  int64_t cin_pad = 0;
  ta.n_ci = 0;
  for (int64_t s = 0; s < nseg; ++s) {
    // 64-channel chunks; the last segment may end in a 32-channel tail (the encoders' 96)
    TORCH_CHECK(in_off[s] % 8 == 0 && (in_cnt[s] % 64 == 0 || (s == nseg - 1 && in_cnt[s] % 32 == 0)),
                "tap-fused wgrad: segments must be multiples of 64 channels (last: of 32)");
    a.seg[s].stride = (int)ins[s].size(3);
    a.seg[s].cnt = (int)in_cnt[s];
    a.seg[s].real = (int)in_cnt[s];
    for (int64_t c = 0; c < in_cnt[s]; c += 64) {
      TORCH_CHECK(ta.n_ci < RAFT_WG_MAX_CI_CHUNKS, "too many input channels");
      ta.ci_seg[ta.n_ci] = (int)s;
      ta.ci_off[ta.n_ci] = (int)c;
      ta.ci_k[ta.n_ci] = (int)(cin_pad + c);
      ta.ci_cnt[ta.n_ci] = (int)std::min<int64_t>(64, in_cnt[s] - c);
      ++ta.n_ci;
    }
    cin_pad += in_cnt[s];
  }
  auto half = [&](const Tensor& t) -> int64_t {
    if (!split) return t.size(3);
    TORCH_CHECK(t.size(3) % 16 == 0, "split fp32 tensors hold two 8-aligned halves");
    return t.size(3) / 2;
  };
  for (int64_t i = 0; i < n0; ++i) {
    const Tensor& g = gs[i];
    check_nhwc(g, B, H, W, "grad", st);
    TORCH_CHECK(g.size(3) == a.g_stride, "all items' grads must share a layout");
    TORCH_CHECK(g_off >= 0 && g_off % 8 == 0 && g_off + (cout + 7) / 8 * 8 <= half(g),
                "grad slice out of range (cout rounded up to 8 channels must fit the row)");
    TORCH_CHECK(g.numel() * 2 < (int64_t(1) << 31), "grad exceeds the 2 GiB buffer-descriptor range");
    it.g[i] = u16(g) + g_off;
    if (split) {
      it.g[n0 + i] = u16(g) + g_off + g.size(3) / 2;   // g_lo x x_hi
      it.g[2 * n0 + i] = u16(g) + g_off;               // g_hi x x_lo
    }
    for (int64_t s = 0; s < nseg; ++s) {
      const Tensor& x = ins[i * nseg + s];
      check_nhwc(x, B, H, W, "wgrad input", st);
      TORCH_CHECK(x.size(3) == a.seg[s].stride, "all items' inputs must share a layout");
      TORCH_CHECK(in_off[s] + in_cnt[s] <= half(x), "segment out of range");
      TORCH_CHECK(x.numel() * 2 < (int64_t(1) << 31), "wgrad input exceeds the 2 GiB buffer-descriptor range");
      it.seg[i][s] = u16(x) + in_off[s];
      if (split) {
        it.seg[n0 + i][s] = u16(x) + in_off[s];
        it.seg[2 * n0 + i][s] = u16(x) + in_off[s] + x.size(3) / 2;
      }
    }
  }
  ta.db_items = split ? (int)(2 * n0) : 0;
  a.cin_pad = (int)cin_pad;
  a.B = (int)B; a.H = (int)H; a.W = (int)W;
  a.KH = (int)kh; a.KW = (int)kw; a.PH = (int)ph; a.PW = (int)pw;
  a.cout = (int)cout;
  // fp32 dw: accumulated (+=); bf16 / fp16 dw: stored (the encoders' 16-bit weight gradients)
  const bool dw_bf16 = dw.scalar_type() == at::kBFloat16 || dw.scalar_type() == at::kHalf;
  TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && (dw_bf16 || dw.scalar_type() == at::kFloat),
              "grad_weight must be a contiguous fp32, bf16 or fp16 GPU tensor");
  const int64_t kpad = kh * kw * cin_pad;
  TORCH_CHECK(dw.dim() == 2 && dw.size(0) == cout && dw.size(1) == kpad, "grad_weight must be (cout, kpad)");
  TORCH_CHECK(kpad % 4 == 0, "packed K must be a multiple of 4");
  a.dw = dw_bf16 ? nullptr : dw.data_ptr<float>();
  ta.dw_bf16 = dw_bf16 ? u16m(dw) : nullptr;
  ta.dw_f16 = dw.scalar_type() == at::kHalf ? 1 : 0;
  a.kpad = (int)kpad;
  ta.bm = (kh == 3 && kw == 3 && cout <= 64) ? 64 : 128;
  ta.n_co = (int)((cout + ta.bm - 1) / ta.bm);
  ta.tiles_x = (int)((W + 7) / 8);
  ta.tiles_per_img = (int)(((H + 7) / 8) * ta.tiles_x);
  ta.chunks_per_item = (int)(B * ta.tiles_per_img);
  ta.total_chunks = (int)(n * ta.chunks_per_item);
  if (splits <= 0) {
    // one full round of equal-sized workgroups (resident per CU: 1 for 3x3 -- 9 x 2 accumulator
    // tiles fill the register file --, 2 for the 5-tap convs, 3 for 1x1); every extra split
    // costs a cout x kpad fp32 partial written and re-read
    const int64_t per_cu = kh * kw == 9 ? (ta.bm == 64 ? 2 : 1) : (kh * kw == 5 ? 2 : 3);
    const int64_t pairs = (int64_t)ta.n_co * ta.n_ci;
    // RAFT_WG_SPLIT_PCT: percentage of that split count (A/B measurements of partial traffic
    // against occupancy; default 100)
    static const int64_t pct = [] {
      const char* e = getenv("RAFT_WG_SPLIT_PCT");
      return e ? std::max<int64_t>(1, atoll(e)) : (int64_t)100;
    }();
    splits = std::max<int64_t>(1, std::min<int64_t>(256 * per_cu * pct / (100 * pairs),
                                                    ta.total_chunks / 8));
  }
  ta.chunks_per_split = (int)((ta.total_chunks + splits - 1) / splits);
  ta.splits = (int)((ta.total_chunks + ta.chunks_per_split - 1) / ta.chunks_per_split);
  TORCH_CHECK(ta.splits < 65536, "too many splits");
  auto fo = dw.options().dtype(at::kFloat);
  Tensor wpart = at::empty({(int64_t)ta.splits * cout * kpad}, fo);
  ta.w_part = wpart.data_ptr<float>();
  float* dbp = nullptr;
  Tensor bpart;
  if (db.has_value() && db->defined()) {
    check_cuda_f32(*db, "grad_bias");
    TORCH_CHECK(db->numel() == cout, "grad_bias size");
    dbp = db->data_ptr<float>();
    bpart = at::empty({(int64_t)ta.splits * cout}, fo);
    ta.db_part = bpart.data_ptr<float>();
  }
  TORCH_CHECK(launch_conv_wgrad_taps(a, it, ta, dbp, cur_stream()), "tap wgrad launch");
}

// Input gradient of a stride-1 "same" conv = the forward kernel on flipped/transposed packed
// weights; the result's channels are scattered over up to 3 fp32 NHWC slices (store or +=).
void conv_dgrad_(const std::vector<Tensor>& ins, const std::vector<int64_t>& in_off,
                 const std::vector<int64_t>& in_cnt, const Tensor& wpk, int64_t kh, int64_t kw,
                 int64_t ph, int64_t pw, int64_t cin_small, double scale,
                 const std::vector<Tensor>& outs, const std::vector<int64_t>& out_off,
                 const std::vector<int64_t>& out_cnt, const std::vector<int64_t>& out_real,
                 const std::vector<int64_t>& out_acc, const std::vector<Tensor>& relu_y,
                 const std::vector<int64_t>& relu_off, const std::vector<int64_t>& gate_mode,
                 const std::vector<Tensor>& gate_t, const std::vector<int64_t>& out_kcin, bool split) {
  TORCH_CHECK(relu_y.size() == relu_off.size(), "relu spec mismatch");
  TORCH_CHECK(out_kcin.empty() || out_kcin.size() == outs.size(), "K-prefix spec mismatch");
  TORCH_CHECK(gate_mode.empty() || gate_mode.size() == outs.size(), "gate spec mismatch");
  TORCH_CHECK(!ins.empty() && ins.size() <= 3 && !outs.empty() && outs.size() <= 3, "1..3 segments");
  TORCH_CHECK(in_off.size() == ins.size() && in_cnt.size() == ins.size(), "input spec mismatch");
  TORCH_CHECK(out_off.size() == outs.size() && out_cnt.size() == outs.size() &&
                  out_real.size() == outs.size() && out_acc.size() == outs.size(),
              "output spec mismatch");
  const int64_t B = ins[0].size(0), H = ins[0].size(1), W = ins[0].size(2);
  c10::DeviceGuard g(ins[0].device());
  ConvFwdArgs a{};
  const at::ScalarType st = op16(ins[0]);
  const int ef16 = st == at::kHalf ? EPI_F16 : 0;
  // split fp32: 16-bit tensors hold [hi | lo] halves (see conv_fwd_); fp32 outputs are plain
  TORCH_CHECK(!split || (st == at::kBFloat16 && cin_small == 0), "split fp32: bf16 pairs, no small-Cin path");
  auto half = [&](const Tensor& t) -> int64_t {
    if (!split) return t.size(3);
    TORCH_CHECK(t.size(3) % 16 == 0, "split fp32 tensors hold two 8-aligned halves");
    return t.size(3) / 2;
  };
  a.nseg = (int)ins.size();
  int64_t cin_pad = 0;
  for (size_t s = 0; s < ins.size(); ++s) {
    check_nhwc(ins[s], B, H, W, "dgrad input", st);
    // a segment may run past the tensor's last channel (a 96-channel tensor in a 128-channel K
    // slot): the kernels read the channels that are not there as zeros
    const int64_t present = std::min<int64_t>(in_cnt[s], half(ins[s]) - in_off[s]);
    TORCH_CHECK(in_off[s] >= 0 && present > 0 && present % 8 == 0 &&
                    (present == in_cnt[s] || cin_small == 0),
                "segment out of range");
    TORCH_CHECK(in_off[s] % 8 == 0 && ins[s].size(3) % 8 == 0, "segments must be 16-byte aligned");
    if (cin_small == 0) TORCH_CHECK(in_cnt[s] % 64 == 0, "segment channels must be a multiple of 64");
    TORCH_CHECK(ins[s].numel() * 2 < (int64_t(1) << 31), "conv input exceeds the 2 GiB buffer-descriptor range");
    a.seg[s].ptr = u16(ins[s]) + in_off[s];
    a.seg[s].stride = (int)ins[s].size(3);
    a.seg[s].cnt = (int)in_cnt[s];
    a.seg[s].real = (int)present;
    cin_pad += in_cnt[s];
  }
  const int64_t cin_seg = cin_pad;  // K-prefix boundaries are in segment channels
  if (split) cin_pad *= 3;           // K thirds [hi | lo | hi]
  a.spl = split ? 1 : 0;
  a.cin_pad = (int)cin_pad;
  a.cin_small = (int)cin_small;
  a.B = (int)B; a.H = (int)H; a.W = (int)W;
  a.KH = (int)kh; a.KW = (int)kw; a.PH = (int)ph; a.PW = (int)pw;
  int64_t cout = 0;
  a.noseg = (int)outs.size();
  for (size_t o = 0; o < outs.size(); ++o) {
    const bool relu_mode = outs[o].scalar_type() != at::kFloat;
    check_nhwc(outs[o], B, H, W, "dgrad output", relu_mode ? st : at::kFloat);
    TORCH_CHECK(outs[o].numel() * outs[o].element_size() < (int64_t(1) << 31),
                "dgrad output exceeds the 2 GiB buffer-descriptor range");
    // the epilogue picks the output segment per 32-column MFMA tile
    TORCH_CHECK(out_cnt[o] % 32 == 0, "dgrad output segments must be multiples of 32 channels");
    TORCH_CHECK(out_real[o] <= out_cnt[o] && out_off[o] >= 0 &&
                    out_off[o] + out_real[o] <= (relu_mode ? half(outs[o]) : outs[o].size(3)),
                "dgrad output slice out of range");
    if (relu_mode && o < relu_off.size() && relu_off[o] < 0) {
      // plain bf16 output (relu_off < 0: no ReLU gate)
      TORCH_CHECK(!out_acc[o], "the bf16 dgrad output cannot accumulate");
      a.oseg[o].ptr = nullptr;
      a.oseg[o].ob = u16m(outs[o]) + out_off[o];
      a.oseg[o].ob_stride = (int)outs[o].size(3);
      a.oseg[o].ry = nullptr;
      a.oseg[o].ry_stride = 0;
    } else if (relu_mode) {
      // bf16 output = relu-gated gradient; relu_y[o] is the forward relu output of these channels
      TORCH_CHECK(o < relu_y.size(), "bf16 dgrad output needs its relu output tensor");
      const Tensor& y = relu_y[o];
      check_nhwc(y, B, H, W, "relu output", st);
      TORCH_CHECK(y.numel() * 2 < (int64_t(1) << 31), "relu output exceeds the 2 GiB descriptor range");
      TORCH_CHECK(relu_off[o] >= 0 && relu_off[o] + out_real[o] <= half(y), "relu output slice out of range");
      TORCH_CHECK(!out_acc[o], "the relu-gated bf16 output cannot accumulate");
      a.oseg[o].ptr = nullptr;
      a.oseg[o].ob = u16m(outs[o]) + out_off[o];
      a.oseg[o].ob_stride = (int)outs[o].size(3);
      a.oseg[o].ry = u16(y) + relu_off[o];
      a.oseg[o].ry_stride = (int)y.size(3);
    } else {
      a.oseg[o].ptr = outs[o].data_ptr<float>() + out_off[o];
      a.oseg[o].ob = nullptr;
      a.oseg[o].ry = nullptr;
    }
    a.oseg[o].stride = (int)outs[o].size(3);
    a.oseg[o].cnt = (int)out_cnt[o];
    a.oseg[o].real = (int)out_real[o];
    a.oseg[o].acc = (int)out_acc[o];
    a.oseg[o].gate = 0;
    cout += out_cnt[o];
  }
  // fused ConvGRU gate backward (see OSeg): 6 tensors per gated segment, in segment order:
  // ga0, ga1, ga2 (bf16: z, q, h | -, r, h | y), gb (bf16), gz (bf16, gate 1), gf1 (fp32)
  size_t gt = 0;
  for (size_t o = 0; o < gate_mode.size(); ++o) {
    const int mode = (int)gate_mode[o];
    if (mode == 0) continue;
    TORCH_CHECK(mode >= 1 && mode <= 3, "gate mode must be 0..3");
    TORCH_CHECK(gt + 6 <= gate_t.size(), "gate tensors missing");
    TORCH_CHECK(outs[o].scalar_type() == at::kFloat, "gated dgrad segment must be fp32");
    TORCH_CHECK(mode == 2 || out_acc[o], "q-gate / relu segments read the accumulated gradient");
    const int real = (int)out_real[o];
    const Tensor& z = gate_t[gt + 0];
    const Tensor& qr = gate_t[gt + 1];
    const Tensor& h = gate_t[gt + 2];
    const Tensor& gbo = gate_t[gt + 3];
    const Tensor& gzo = gate_t[gt + 4];
    const Tensor& gf1 = gate_t[gt + 5];
    gt += 6;
    for (const Tensor* t : {&z, &qr, &h}) {
      check_nhwc(*t, B, H, W, "gate input", st);
      TORCH_CHECK(t->size(3) == z.size(3) && half(*t) >= real, "gate inputs must share a layout");
      TORCH_CHECK(t->numel() * 2 < (int64_t(1) << 31), "gate input exceeds the 2 GiB descriptor range");
    }
    for (const Tensor* t : {&gbo, &gzo}) {
      check_nhwc(*t, B, H, W, "gate output", st);
      TORCH_CHECK(t->numel() * 2 < (int64_t(1) << 31), "gate output exceeds the 2 GiB descriptor range");
    }
    TORCH_CHECK(half(gbo) >= (mode == 2 ? 2 * real : real), "gate d-pre output too narrow");
    TORCH_CHECK(mode != 1 || half(gzo) >= real, "gate d-pre-z output too narrow");
    check_nhwc(gf1, B, H, W, "gate state gradient", at::kFloat);
    TORCH_CHECK(gf1.size(3) >= real && gf1.numel() * 4 < (int64_t(1) << 31), "gate state gradient");
    a.oseg[o].gate = mode;
    a.oseg[o].ga0 = u16(z);
    a.oseg[o].ga1 = u16(qr);
    a.oseg[o].ga2 = u16(h);
    a.oseg[o].ga_stride = (int)z.size(3);
    a.oseg[o].gb = u16m(gbo);
    a.oseg[o].gb_stride = (int)gbo.size(3);
    a.oseg[o].gz = u16m(gzo);
    a.oseg[o].gz_stride = (int)gzo.size(3);
    a.oseg[o].gf1 = gf1.data_ptr<float>();
    a.oseg[o].gf_stride = (int)gf1.size(3);
  }
  // per-segment K prefixes: a prefix must end on an input-segment boundary (multiple of 64)
  a.kprefix = 0;
  for (size_t o = 0; o < out_kcin.size(); ++o) {
    const int64_t kc = out_kcin[o];
    // split fp32: the K thirds interleave hi / lo, so a prefix is no longer contiguous -- the
    // full K runs (the packed weight is zero past the prefix anyway)
    if (kc == 0 || kc == cin_seg || split) continue;
    int64_t acc = 0;
    bool on_boundary = false;
    for (size_t s2 = 0; s2 < ins.size(); ++s2) { acc += in_cnt[s2]; on_boundary = on_boundary || acc == kc; }
    TORCH_CHECK(kc > 0 && kc < cin_seg && kc % 64 == 0 && on_boundary && cin_small == 0,
                "out_kcin must end on an input segment boundary");
    a.oseg[o].kcin = (int)kc;
    a.kprefix = 1;
  }
  TORCH_CHECK(gt == gate_t.size(), "unused gate tensors");
  a.cout = (int)cout;
  const int bn = (cout % 128 == 0) ? 128 : 64;
  TORCH_CHECK(wpk.is_cuda() && wpk.is_contiguous() && wpk.scalar_type() == st && wpk.dim() == 2,
              "packed weight must be a contiguous (Npad, Kpad) tensor of the operand dtype");
  const int64_t kneed = cin_small ? ((kh * kw * cin_small + 63) / 64) * 64 : kh * kw * cin_pad;
  TORCH_CHECK(wpk.size(1) == kneed, "packed dgrad weight K mismatch: ", wpk.size(1), " vs ", kneed);
  TORCH_CHECK(wpk.size(0) >= cout, "packed dgrad weight has too few rows");
  a.wpk = u16(wpk);
  a.kpad = (int)wpk.size(1);
  a.bias = nullptr;
  a.scale = (float)scale;
  bool any_gate = false;
  for (int o = 0; o < a.noseg; ++o) any_gate = any_gate || a.oseg[o].gate != 0;
  TORCH_CHECK(!(any_gate && cin_small), "gated dgrad needs the 64-channel K path");
  TORCH_CHECK(!ef16 || cin_small == 0, "fp16 operands: no small-Cin path");
  TORCH_CHECK(launch_conv_fwd(a, (any_gate ? EPI_DGRAD_GATE : EPI_DGRAD) | ef16 | (split ? EPI_SPL : 0), bn, cin_small != 0, cur_stream()),
              "dgrad launch");
}

// ------------------------------------------------------------------ encoder norm + activation
// Tensors are NCHW-shaped channels_last bf16, fp16 under fp16 autocast, or fp32 (the fp32
// schedule) -- the memory is NHWC; every activation tensor of one call has the dtype st of its
// first.
at::ScalarType opnorm(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf ||
                  t.scalar_type() == at::kFloat,
              "encoder norm tensors must be bfloat16, float16 or float32, got ", t.scalar_type());
  return t.scalar_type();
}
// the launchers' storage-type flag: 0 bf16, 1 fp16, 2 fp32
int norm_ty(at::ScalarType st) { return st == at::kHalf ? 1 : (st == at::kFloat ? 2 : 0); }
void check_cl16(at::ScalarType st, const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == st && t.dim() == 4, name,
              ": must be a 4-D GPU tensor of dtype ", st);
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, ": must be channels_last");
  TORCH_CHECK(t.size(1) % 8 == 0 && t.size(1) <= 256, name, ": channels must be a multiple of 8, <= 256");
}
// optional split-bf16 operand buffer of an fp32 NCHW-shaped channels_last tensor x: contiguous
// (N, H, W, 2 spad) bf16 with spad >= C a multiple of 8 -> (pointer, spad)
std::pair<uint16_t*, int> opt_split(const c10::optional<Tensor>& t, const Tensor& x, const char* name) {
  if (!t.has_value() || !t->defined()) return {nullptr, 0};
  TORCH_CHECK(x.scalar_type() == at::kFloat, name, ": split operands are for fp32 tensors");
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 4 &&
                  t->size(0) == x.size(0) && t->size(1) == x.size(2) && t->size(2) == x.size(3) &&
                  t->size(3) % 16 == 0 && t->size(3) / 2 >= x.size(1),
              name, ": must be a contiguous (N, H, W, 2 spad) bf16 tensor, spad >= C");
  return {u16m(*t), (int)(t->size(3) / 2)};
}
const float* opt_f32(const c10::optional<Tensor>& t, int64_t n, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_cuda_f32(*t, name);
  TORCH_CHECK(t->numel() == n, name, ": size mismatch");
  return t->data_ptr<float>();
}

// y = act(norm(x + cbias)) [+ res, relu]; returns (mean, invstd) for the backward
std::vector<Tensor> norm_fwd_(const Tensor& x, int64_t mode, int64_t relu,
                              const c10::optional<Tensor>& gamma, const c10::optional<Tensor>& beta,
                              const c10::optional<Tensor>& cbias,
                              const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rvar,
                              double momentum, double eps, const c10::optional<Tensor>& res,
                              const Tensor& y, const c10::optional<Tensor>& ysplit,
                              const c10::optional<Tensor>& tstats, int64_t tiles) {
  const at::ScalarType st = opnorm(x);
  check_cl16(st, x, "x");
  check_cl16(st, y, "y");
  TORCH_CHECK(y.sizes() == x.sizes(), "y shape");
  TORCH_CHECK(mode >= 0 && mode <= 3, "mode");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  c10::DeviceGuard g(x.device());
  const float* gp = opt_f32(gamma, C, "gamma");
  const float* bp = opt_f32(beta, C, "beta");
  const float* cb = opt_f32(cbias, C, "conv bias");
  float* rm = const_cast<float*>(opt_f32(rmean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(rvar, C, "running_var"));
  if (mode == 2) TORCH_CHECK(rm && rv, "eval batch norm needs running stats");
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_cl16(st, *res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res shape");
    rp = u16(*res);
  }
  const int groups = mode == 0 ? (int)N : 1;
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({groups, C}, fo), invstd = at::empty({groups, C}, fo);
  Tensor scale = at::empty({N, C}, fo), shift = at::empty({N, C}, fo);
  const uint16_t* xp = u16(x);
  int ppb = 0, nblk = 0;
  Tensor part;
  const bool tiled = mode <= 1 && tstats.has_value() && tstats->defined();
  if (tiled) {
    // the producing conv's per-tile statistics: no statistics pass over x
    check_cuda_f32(*tstats, "tstats");
    TORCH_CHECK(tiles > 0 && tstats->is_contiguous() && tstats->numel() == N * tiles * 4 * C,
                "tstats must be a contiguous (N * tiles, 4, C) fp32 tensor");
    launch_norm_finalize_tiled(tstats->data_ptr<float>(), mode == 0 ? (int)tiles : (int)(N * tiles),
                               (int)N, (int)HW, (int)C, (int)mode, gp, bp, cb, rm, rv,
                               (float)momentum, (float)eps, mean.data_ptr<float>(),
                               invstd.data_ptr<float>(), scale.data_ptr<float>(),
                               shift.data_ptr<float>(), cur_stream());
  } else {
    if (mode <= 1) {
      nblk = encoder_norm_blocks(mode == 0 ? HW : N * HW, (int)C, groups, &ppb);
      part = at::empty({groups * (nblk + 1) * 2 * C}, fo);  // partials + per-group sums
      launch_norm_stats(xp, (int)N, (int)HW, (int)C, mode == 0, part.data_ptr<float>(), nblk, ppb,
                        norm_ty(st), cur_stream());
    }
    launch_norm_finalize(mode <= 1 ? part.data_ptr<float>() : nullptr, xp, (int)N, (int)HW, (int)C,
                         (int)mode, nblk, gp, bp, cb, rm, rv, (float)momentum, (float)eps,
                         mean.data_ptr<float>(), invstd.data_ptr<float>(), scale.data_ptr<float>(),
                         shift.data_ptr<float>(), norm_ty(st), cur_stream());
  }
  const auto ys = opt_split(ysplit, x, "ysplit");
  launch_norm_apply(xp, scale.data_ptr<float>(), shift.data_ptr<float>(), (int)N, (int)HW, (int)C,
                    (int)relu, rp, u16m(y), norm_ty(st), cur_stream(), ys.first, ys.second);
  return {mean, invstd};
}

// dx (bf16) and += parameter grads; y = the forward output when relu (mask), else ignored
void norm_bwd_(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& y,
               const Tensor& mean, const Tensor& invstd, int64_t mode, int64_t relu, const c10::optional<Tensor>& gamma,
               const c10::optional<Tensor>& beta, const c10::optional<Tensor>& dgamma,
               const c10::optional<Tensor>& dbeta, const c10::optional<Tensor>& dcbias,
               const Tensor& dx, const c10::optional<Tensor>& dy2, const c10::optional<Tensor>& yres,
               const c10::optional<Tensor>& gout, const c10::optional<Tensor>& dxsplit) {
  const at::ScalarType st = opnorm(dy);
  check_cl16(st, dy, "dy");
  check_cl16(st, x, "x");
  check_cl16(st, dx, "dx");
  TORCH_CHECK(dy.sizes() == x.sizes() && dx.sizes() == x.sizes(), "shapes");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  const int groups = mode == 0 ? (int)N : 1;
  check_cuda_f32(mean, "mean");
  check_cuda_f32(invstd, "invstd");
  TORCH_CHECK(mean.numel() == groups * C && invstd.numel() == groups * C, "stat shapes");
  c10::DeviceGuard g(x.device());
  const float* gp = opt_f32(gamma, C, "gamma");
  const float* bp = opt_f32(beta, C, "beta");
  float* dg = const_cast<float*>(opt_f32(dgamma, C, "dgamma"));
  float* db = const_cast<float*>(opt_f32(dbeta, C, "dbeta"));
  float* dc = const_cast<float*>(opt_f32(dcbias, C, "dcbias"));
  int ppb = 0;
  const int nblk = encoder_norm_blocks(mode == 0 ? HW : N * HW, (int)C, groups, &ppb);
  auto fo = x.options().dtype(at::kFloat);
  Tensor part = at::empty({groups * (nblk + 1) * 3 * C}, fo);  // partials + per-group sums
  Tensor coef = at::empty({groups, 5, C}, fo);  // A, B', C', scale, shift per (group, c), SoA
  const uint16_t* yp = nullptr;
  if (y.has_value() && y->defined()) {
    check_cl16(st, *y, "y");
    TORCH_CHECK(y->sizes() == x.sizes(), "y shape");
    yp = u16(*y);
  }
  // fused block-end ReLU: g = (dy [+ dy2]) * [yres > 0] -> gout, the norm backward runs on g
  const uint16_t *d2 = nullptr, *yr = nullptr;
  uint16_t* go = nullptr;
  if (yres.has_value() && yres->defined()) {
    check_cl16(st, *yres, "yres");
    TORCH_CHECK(gout.has_value() && gout->defined(), "yres needs gout");
    check_cl16(st, *gout, "gout");
    TORCH_CHECK(yres->sizes() == x.sizes() && gout->sizes() == x.sizes(), "yres / gout shape");
    yr = u16(*yres);
    go = u16m(*gout);
    if (dy2.has_value() && dy2->defined()) {
      check_cl16(st, *dy2, "dy2");
      TORCH_CHECK(dy2->sizes() == x.sizes(), "dy2 shape");
      d2 = u16(*dy2);
    }
  } else {
    TORCH_CHECK(!(dy2.has_value() && dy2->defined()), "dy2 needs yres");
  }
  const auto dxs = opt_split(dxsplit, x, "dxsplit");
  launch_norm_bwd(u16(dy),
                  u16(x), yp, mean.data_ptr<float>(),
                  invstd.data_ptr<float>(), (int)N, (int)HW, (int)C, (int)mode, (int)relu, gp, bp,
                  part.data_ptr<float>(), nblk, ppb, coef.data_ptr<float>(), dg, db, dc,
                  u16m(dx), d2, yr, go, norm_ty(st), cur_stream(), dxs.first, dxs.second);
}

// context-encoder output: cnet (B,C,H,W) channels_last bf16 / fp16 -> h (B,H,W,hdim) =
// tanh(cnet[:, :hdim]), x (B,H,W,C-hdim) = relu(cnet[:, hdim:]), both contiguous NHWC
void check_nhwc_like(const Tensor& t, const Tensor& cnet, int64_t c, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == cnet.scalar_type() && t.is_contiguous() && t.dim() == 4 &&
                  t.size(0) == cnet.size(0) && t.size(1) == cnet.size(2) && t.size(2) == cnet.size(3) &&
                  t.size(3) == c,
              name, ": must be a contiguous (B,H,W,", c, ") tensor of the input's dtype");
}
void ctx_act_(const Tensor& cnet, int64_t hdim, const Tensor& h, const Tensor& x) {
  const at::ScalarType st = opnorm(cnet);
  TORCH_CHECK(st != at::kFloat, "ctx_act: bf16 / fp16 only");
  check_cl16(st, cnet, "cnet");
  const int64_t C = cnet.size(1);
  TORCH_CHECK(hdim % 8 == 0 && hdim > 0 && hdim < C, "ctx_act: hdim must be a multiple of 8 below C");
  check_nhwc_like(h, cnet, hdim, "h");
  check_nhwc_like(x, cnet, C - hdim, "x");
  c10::DeviceGuard g(cnet.device());
  launch_ctx_act(u16(cnet), cnet.size(0) * cnet.size(2) * cnet.size(3), (int)C, (int)hdim, u16m(h), u16m(x),
                 norm_ty(st), cur_stream());
}
void ctx_act_bwd_(const c10::optional<Tensor>& gh, const c10::optional<Tensor>& gx, const Tensor& h,
                  const Tensor& x, const Tensor& gin) {
  const at::ScalarType st = opnorm(gin);
  TORCH_CHECK(st != at::kFloat, "ctx_act_bwd: bf16 / fp16 only");
  check_cl16(st, gin, "gin");
  const int64_t C = gin.size(1), hdim = h.size(3);
  TORCH_CHECK(hdim % 8 == 0 && hdim > 0 && hdim < C, "ctx_act_bwd: hdim");
  check_nhwc_like(h, gin, hdim, "h");
  check_nhwc_like(x, gin, C - hdim, "x");
  const uint16_t *ghp = nullptr, *gxp = nullptr;
  if (gh.has_value() && gh->defined()) {
    check_nhwc_like(*gh, gin, hdim, "gh");
    ghp = u16(*gh);
  }
  if (gx.has_value() && gx->defined()) {
    check_nhwc_like(*gx, gin, C - hdim, "gx");
    gxp = u16(*gx);
  }
  c10::DeviceGuard g(gin.device());
  launch_ctx_act_bwd(ghp, gxp, u16(h), u16(x), gin.size(0) * gin.size(2) * gin.size(3), (int)C, (int)hdim,
                     u16m(gin), norm_ty(st), cur_stream());
}

void add_relu_(const Tensor& a, const Tensor& b, const Tensor& out) {
  const at::ScalarType st = opnorm(a);
  check_cl16(st, a, "a");
  check_cl16(st, b, "b");
  check_cl16(st, out, "out");
  TORCH_CHECK(a.sizes() == b.sizes() && out.sizes() == a.sizes(), "shapes");
  c10::DeviceGuard g(a.device());
  launch_add_relu(u16(a),
                  u16(b),
                  u16m(out), a.numel(), norm_ty(st), cur_stream());
}

// out (2B,3,H,W) channels_last = 2 * ([a ; b] / 255) - 1 in out's dtype; a, b (B,3,H,W) fp32
void image_prep_(const Tensor& a, const Tensor& b, const Tensor& out) {
  check_cuda_f32(a, "image a");
  check_cuda_f32(b, "image b");
  TORCH_CHECK(a.dim() == 4 && a.size(1) == 3 && a.sizes() == b.sizes(), "images must be (B,3,H,W)");
  TORCH_CHECK(a.device() == b.device() && out.device() == a.device(), "image_prep: devices");
  const int64_t B = a.size(0), H = a.size(2), W = a.size(3);
  TORCH_CHECK(out.dim() == 4 && out.size(0) == 2 * B && out.size(1) == 3 && out.size(2) == H &&
              out.size(3) == W && out.is_contiguous(at::MemoryFormat::ChannelsLast),
              "image_prep: out must be a channels_last (2B,3,H,W) tensor");
  const at::ScalarType ot = out.scalar_type();
  TORCH_CHECK(ot == at::kBFloat16 || ot == at::kHalf || ot == at::kFloat, "image_prep: out dtype");
  c10::DeviceGuard gd(a.device());
  TORCH_CHECK(launch_image_prep(a.data_ptr<float>(), b.data_ptr<float>(), out.data_ptr(), (int)B, H * W,
                                ot == at::kBFloat16 ? 0 : (ot == at::kHalf ? 1 : 2), cur_stream()),
              "image_prep launch");
}

// out[i] = cast(srcs[k][off]) for idx[i] = k << 26 | off (k = 63: zero); srcs contiguous GPU
// tensors of one dtype and device, out 1-D with idx.numel() elements: fp32 sources -> bf16 /
// fp16 / fp32 out, or bf16 / fp16 sources -> fp32 out
void gather_cast_(const std::vector<Tensor>& srcs, const Tensor& idx, const Tensor& out, int64_t lo_from) {
  TORCH_CHECK(!srcs.empty() && (int64_t)srcs.size() <= RAFT_GATHER_MAX, "gather: 1..",
              RAFT_GATHER_MAX, " sources");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kInt && idx.is_contiguous() && idx.dim() == 1,
              "gather: idx must be a contiguous 1-D int32 GPU tensor");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.numel() == idx.numel(),
              "gather: out must be contiguous with idx.numel() elements");
  const at::ScalarType ot = out.scalar_type();
  TORCH_CHECK(ot == at::kBFloat16 || ot == at::kHalf || ot == at::kFloat, "gather: out dtype");
  const at::ScalarType it = srcs[0].scalar_type();
  TORCH_CHECK(it == at::kBFloat16 || it == at::kHalf || it == at::kFloat, "gather: source dtype");
  TORCH_CHECK(it == at::kFloat || ot == at::kFloat, "gather: 16-bit sources need an fp32 output");
  GatherSrcs gs{};
  gs.n = (int)srcs.size();
  // lo_from >= 0: sources [lo_from, n) give split-fp32 residuals (fp32 sources, bf16 output)
  gs.lo_from = lo_from < 0 ? RAFT_GATHER_MAX : (int)lo_from;
  TORCH_CHECK(lo_from < 0 || (it == at::kFloat && ot == at::kBFloat16), "gather: residuals need fp32 -> bf16");
  for (int k = 0; k < gs.n; ++k) {
    TORCH_CHECK(srcs[k].is_cuda() && srcs[k].scalar_type() == it && srcs[k].is_contiguous() &&
                srcs[k].device() == idx.device() && srcs[k].numel() <= (1 << 26),
                "gather: sources must be contiguous GPU tensors of one dtype and device");
    gs.p[k] = srcs[k].data_ptr();
  }
  TORCH_CHECK(out.device() == idx.device(), "gather: devices");
  auto ty = [](at::ScalarType t) { return t == at::kBFloat16 ? 0 : (t == at::kHalf ? 1 : 2); };
  c10::DeviceGuard gd(idx.device());
  TORCH_CHECK(launch_gather_cast(gs, idx.data_ptr<int32_t>(), out.data_ptr(), idx.numel(), ty(it),
                                 ty(ot), cur_stream()),
              "gather launch");
}

void relu_mask_(const Tensor& dy, const Tensor& y, const Tensor& g, const c10::optional<Tensor>& dy2) {
  const at::ScalarType st = opnorm(dy);
  check_cl16(st, dy, "dy");
  check_cl16(st, y, "y");
  check_cl16(st, g, "g");
  TORCH_CHECK(dy.sizes() == y.sizes() && g.sizes() == y.sizes(), "shapes");
  const uint16_t* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    check_cl16(st, *dy2, "dy2");
    TORCH_CHECK(dy2->sizes() == y.sizes(), "dy2 shape");
    d2 = u16(*dy2);
  }
  c10::DeviceGuard gd(y.device());
  launch_relu_mask(u16(dy), d2,
                   u16(y),
                   u16m(g), y.numel(), norm_ty(st), cur_stream());
}

// ------------------------------------------------------------------ update-block elementwise
const uint16_t* bf16p(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr<at::BFloat16>()); }
uint16_t* bf16m(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr<at::BFloat16>()); }

void check_pc(const Tensor& t, int64_t P, int64_t C, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == st, name, ": wrong device/dtype/layout");
  TORCH_CHECK(t.numel() == P * C, name, ": expected ", P, " x ", C, " elements");
}

// out[:, o_off:o_off+C] (bf16) = g[:, g_off:g_off+C] * scale * [y[:, y_off:] > 0]
// stride-1 3x3 conv, 64 -> 64 channels, NHWC bf16 (the encoders' layer1; forward, or the input
// gradient with the adjoint weight pack)
// ---- encoder stem conv (stem_conv.hip): 7x7, stride 2, pad 3, 3 -> C (64 / 32) channels.
// x (B,H,W,3) and out (B,Ho,Wo,C) contiguous NHWC 16-bit; w the (C,7,7,3)-ordered weight (the
// memory of a channels_last (C,3,7,7) weight)
int device_cus() {
  static const int cus = [] {
    hipDeviceProp_t p{};
    int dev = 0;
    (void)hipGetDevice(&dev);
    return hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
  }();
  return cus;
}
void stem_checks(const Tensor& x, at::ScalarType st, int64_t& B, int64_t& H, int64_t& W, int64_t& Ho, int64_t& Wo) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(3) == 3 && x.is_contiguous() && x.scalar_type() == st,
              "stem conv: x must be a contiguous (B,H,W,3) 16-bit NHWC tensor");
  B = x.size(0), H = x.size(1), W = x.size(2);
  Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  TORCH_CHECK(H * W * 6 < (int64_t(1) << 31), "stem conv: image too large");
}
void stem_conv_fwd_(const Tensor& x, const Tensor& w, const Tensor& out) {
  const at::ScalarType st = op16(x);
  int64_t B, H, W, Ho, Wo;
  stem_checks(x, st, B, H, W, Ho, Wo);
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && w.scalar_type() == st && w.dim() == 4 &&
                  w.size(1) == 7 && w.size(2) == 7 && w.size(3) == 3 && (w.size(0) == 64 || w.size(0) == 32),
              "stem conv: w must be a contiguous (C,7,7,3) 16-bit tensor, C = 64 or 32");
  const int64_t C = w.size(0);
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.scalar_type() == st && out.dim() == 4 &&
                  out.size(0) == B && out.size(1) == Ho && out.size(2) == Wo && out.size(3) == C,
              "stem conv: out must be a contiguous (B,Ho,Wo,C) tensor of x's dtype");
  TORCH_CHECK(Ho * Wo * C * 2 < (int64_t(1) << 31), "stem conv: output too large");
  c10::DeviceGuard gd(x.device());
  const int tiles = stem_conv_tiles((int)B, (int)Ho, (int)Wo);
  const int grid = std::min(tiles, 2 * device_cus());
  TORCH_CHECK(launch_stem_conv_fwd(u16(x), u16(w), u16m(out), (int)B, (int)H, (int)W, (int)Ho, (int)Wo,
                                   (int)C, grid, st == at::kHalf, cur_stream()),
              "stem conv forward launch");
}
// -> dw (C,7,7,3), x's dtype: the weight gradient for the output gradient gy (B,Ho,Wo,C)
Tensor stem_conv_wgrad(const Tensor& x, const Tensor& gy) {
  const at::ScalarType st = op16(x);
  int64_t B, H, W, Ho, Wo;
  stem_checks(x, st, B, H, W, Ho, Wo);
  TORCH_CHECK(gy.is_cuda() && gy.is_contiguous() && gy.scalar_type() == st && gy.dim() == 4 &&
                  gy.size(0) == B && gy.size(1) == Ho && gy.size(2) == Wo &&
                  (gy.size(3) == 64 || gy.size(3) == 32),
              "stem conv: gy must be a contiguous (B,Ho,Wo,C) tensor of x's dtype, C = 64 or 32");
  const int64_t C = gy.size(3);
  TORCH_CHECK(Ho * Wo * C * 2 < (int64_t(1) << 31), "stem conv: output gradient too large");
  c10::DeviceGuard gd(x.device());
  const int tiles = stem_conv_tiles((int)B, (int)Ho, (int)Wo);
  // 3 workgroups per CU (50 KB of LDS each): more tile loads in flight
  const int grid = std::min(tiles, 3 * device_cus());
  Tensor part = at::empty({grid, C, 224}, x.options().dtype(at::kFloat));
  Tensor dw = at::empty({C, 7, 7, 3}, x.options());
  TORCH_CHECK(launch_stem_conv_wgrad(u16(x), u16(gy), part.data_ptr<float>(), u16m(dw), (int)B, (int)H,
                                     (int)W, (int)Ho, (int)Wo, (int)C, grid, st == at::kHalf, cur_stream()),
              "stem conv weight-gradient launch");
  return dw;
}

// part (optional): the norm statistics of the output per 8 x 16 tile, (B * tiles, 4, 64) fp32
// (see launch_conv_enc64), for norm_fwd_'s tstats
void conv_enc64_(const Tensor& x, const Tensor& wpk, const Tensor& out, const c10::optional<Tensor>& part) {
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 64, "x must be (B,H,W,64)");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2);
  const at::ScalarType st = op16(x);
  check_nhwc(x, B, H, W, "conv_enc64 input", st);
  check_nhwc(out, B, H, W, "conv_enc64 output", st);
  TORCH_CHECK(out.size(3) == 64, "out must be (B,H,W,64)");
  TORCH_CHECK(wpk.is_cuda() && wpk.is_contiguous() && wpk.scalar_type() == st &&
                  wpk.dim() == 2 && wpk.size(0) == 64 && wpk.size(1) == 9 * 64,
              "packed weight must be a contiguous (64, 576) tensor of the operand dtype");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31) && H * W * 128 < (int64_t(1) << 31), "conv_enc64: input too large");
  c10::DeviceGuard gd(x.device());
  static const int cus = [] {
    hipDeviceProp_t p{};
    int dev = 0;
    (void)hipGetDevice(&dev);
    return hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
  }();
  float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    check_cuda_f32(*part, "conv_enc64 part");
    TORCH_CHECK(part->is_contiguous() &&
                    part->numel() == B * conv_enc64_tiles((int)H, (int)W) * 4 * 64,
                "conv_enc64 part must be a contiguous (B * tiles, 4, 64) fp32 tensor");
    pp = part->data_ptr<float>();
  }
  TORCH_CHECK(launch_conv_enc64(u16(x), u16(wpk), u16m(out), (int)B, (int)H, (int)W, cus,
                                st == at::kHalf, cur_stream(), pp),
              "conv_enc64 launch failed");
}

void split_hilo_(const Tensor& x, const Tensor& out) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4, "x: fp32 (B,C,H,W)");
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  check_nhwc(out, B, H, W, "split_hilo out", at::kBFloat16);
  const int64_t cp = out.size(3) / 2;
  TORCH_CHECK(out.size(3) % 2 == 0 && cp % 8 == 0 && cp >= C, "out must be (B,H,W,2cp), cp >= C, cp % 8 == 0");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31) && out.numel() < (int64_t(1) << 31), "split_hilo: tensor too large");
  c10::DeviceGuard gd(x.device());
  launch_split_hilo(x.data_ptr<float>(), x.stride(0), x.stride(1), x.stride(2), x.stride(3), (int)B,
                    (int)C, (int)H, (int)W, (int)cp, bf16m(out), cur_stream());
}

void relu_bwd_(const Tensor& g, int64_t g_off, const c10::optional<Tensor>& y, int64_t y_off,
               const Tensor& out, int64_t o_off, int64_t C, double scale, bool split) {
  TORCH_CHECK(g.is_cuda() && g.is_contiguous() && g.scalar_type() == at::kFloat && g.dim() == 4, "g: fp32 NHWC");
  const int64_t B = g.size(0), H = g.size(1), W = g.size(2), P = B * H * W;
  TORCH_CHECK(g_off + C <= g.size(3), "g slice");
  const at::ScalarType st = op16(out);   // bf16, or fp16 under fp16 autocast
  TORCH_CHECK(!split || st == at::kBFloat16, "split fp32: bf16 [hi | lo] pairs");
  check_nhwc(out, B, H, W, "relu_bwd out", st);
  // split fp32: offsets / C index the hi half, the lo half is the row's second half
  const int64_t ow = split ? out.size(3) / 2 : out.size(3);
  TORCH_CHECK(!split || out.size(3) % 2 == 0, "split out: two halves");
  TORCH_CHECK(o_off + C <= ow, "out slice");
  const uint16_t* yp = nullptr;
  int ys = 0;
  if (y.has_value() && y->defined()) {
    check_nhwc(*y, B, H, W, "relu_bwd y", st);
    TORCH_CHECK(!split || y->size(3) % 2 == 0, "split y: two halves");
    TORCH_CHECK(y_off + C <= (split ? y->size(3) / 2 : y->size(3)), "y slice");
    yp = u16(*y) + y_off;
    ys = (int)y->size(3);
  }
  c10::DeviceGuard gd(g.device());
  launch_relu_bwd(g.data_ptr<float>() + g_off, (int)g.size(3), yp, ys, u16m(out) + o_off,
                  (int)out.size(3), (int)P, (int)C, (float)scale, cur_stream(),
                  split ? 2 : (st == at::kHalf ? 1 : 0));
}

// split fp32 (bf16 [hi | lo] rows of twice the width) is recognised by the 16-bit tensors' width
void gru_q_bwd_(const Tensor& dh, const Tensor& z, const Tensor& q, const Tensor& hprev,
                const Tensor& dpre_q, const Tensor& dz, const Tensor& dhprev) {
  TORCH_CHECK(dh.dim() == 4 && z.dim() == 4, "dh, z must be (B,H,W,hd)");
  const int64_t P = dh.size(0) * dh.size(1) * dh.size(2), hd = dh.size(3);
  const at::ScalarType st = op16(z);   // bf16, or fp16 under fp16 autocast
  const bool split = st == at::kBFloat16 && z.size(3) == 2 * hd;
  const int64_t w = split ? 2 * hd : hd;
  check_pc(dh, P, hd, at::kFloat, "dh");
  check_pc(z, P, w, st, "z");
  check_pc(q, P, w, st, "q");
  check_pc(hprev, P, w, st, "hprev");
  check_pc(dpre_q, P, w, st, "dpre_q");
  check_pc(dz, P, hd, at::kFloat, "dz");
  check_pc(dhprev, P, hd, at::kFloat, "dhprev");
  c10::DeviceGuard gd(dh.device());
  launch_gru_q_bwd(dh.data_ptr<float>(), u16(z), u16(q), u16(hprev), u16m(dpre_q),
                   dz.data_ptr<float>(), dhprev.data_ptr<float>(), (int)P, (int)hd, cur_stream(),
                   split ? 2 : (st == at::kHalf ? 1 : 0));
}

void gru_zr_bwd_(const Tensor& drh, const Tensor& dz, const Tensor& z, const Tensor& r,
                 const Tensor& hprev, const Tensor& dpre_zr, const Tensor& dhprev) {
  TORCH_CHECK(drh.dim() == 4 && z.dim() == 4, "drh, z must be (B,H,W,hd)");
  const int64_t P = drh.size(0) * drh.size(1) * drh.size(2), hd = drh.size(3);
  const at::ScalarType st = op16(z);
  const bool split = st == at::kBFloat16 && z.size(3) == 2 * hd;
  const int64_t w = split ? 2 * hd : hd;
  check_pc(drh, P, hd, at::kFloat, "drh");
  check_pc(dz, P, hd, at::kFloat, "dz");
  check_pc(z, P, w, st, "z");
  check_pc(r, P, w, st, "r");
  check_pc(hprev, P, w, st, "hprev");
  check_pc(dpre_zr, P, 2 * w, st, "dpre_zr");
  check_pc(dhprev, P, hd, at::kFloat, "dhprev");
  c10::DeviceGuard gd(drh.device());
  launch_gru_zr_bwd(drh.data_ptr<float>(), dz.data_ptr<float>(), u16(z), u16(r), u16(hprev),
                    u16m(dpre_zr), dhprev.data_ptr<float>(), (int)P, (int)hd, cur_stream(),
                    split ? 2 : (st == at::kHalf ? 1 : 0));
}

// out = sum(ins) (+ carry): n <= RAFT_SUM_MAX same-shape contiguous bf16 tensors, fp32 accumulation,
// out bf16 or fp32 of the same shape
void sum_bf16_(const std::vector<Tensor>& ins, const c10::optional<Tensor>& carry, const Tensor& out) {
  TORCH_CHECK(!ins.empty() && ins.size() <= RAFT_SUM_MAX, "1..", RAFT_SUM_MAX, " summands");
  const int64_t numel = out.numel();
  TORCH_CHECK(numel % 8 == 0, "sum_bf16_: numel must be a multiple of 8");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() &&
                  (out.scalar_type() == op16(ins[0]) || out.scalar_type() == at::kFloat),
              "sum_bf16_: out must be a contiguous GPU tensor of the summands' dtype or fp32");
  BfPtrs p{};
  for (size_t k = 0; k < ins.size(); ++k) {
    TORCH_CHECK(ins[k].is_cuda() && ins[k].is_contiguous() && ins[k].scalar_type() == ins[0].scalar_type() &&
                    ins[k].numel() == numel && ins[k].device() == out.device(),
                "sum_bf16_: summands must be contiguous 16-bit tensors of one dtype and the output's size");
    p.p[k] = u16(ins[k]);
    TORCH_CHECK(reinterpret_cast<uintptr_t>(p.p[k]) % 16 == 0, "sum_bf16_: summands must be 16-byte aligned");
  }
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "sum_bf16_: out must be 16-byte aligned");
  const float* cp = nullptr;
  if (carry.has_value() && carry->defined()) {
    check_cuda_f32(*carry, "carry");
    TORCH_CHECK(carry->numel() == numel, "carry size");
    cp = carry->data_ptr<float>();
    TORCH_CHECK(reinterpret_cast<uintptr_t>(cp) % 16 == 0, "sum_bf16_: carry must be 16-byte aligned");
  }
  c10::DeviceGuard gd(out.device());
  launch_sum_bf16(p, (int)ins.size(), cp, out.data_ptr(), out.scalar_type() == at::kFloat, numel,
                  ins[0].scalar_type() == at::kHalf, cur_stream());
}

// flow (B,2,H,W) fp32 -> flowb (B,H,W,8) bf16 [fx, fy, 0...]; optionally slot[..., off:off+2] = flow
void flow_prep_(const Tensor& flow, const Tensor& flowb, const c10::optional<Tensor>& slot,
                int64_t slot_off) {
  check_cuda_f32(flow, "flow");
  TORCH_CHECK(flow.dim() == 4 && flow.size(1) == 2, "flow must be (B,2,H,W)");
  const int64_t B = flow.size(0), H = flow.size(2), W = flow.size(3);
  check_nhwc(flowb, B, H, W, "flowb", at::kBFloat16);
  TORCH_CHECK(flowb.size(3) == 8, "flowb must have 8 channels");
  uint16_t* sp = nullptr;
  int ss = 0;
  if (slot.has_value() && slot->defined()) {
    check_nhwc(*slot, B, H, W, "slot", at::kBFloat16);
    TORCH_CHECK(slot_off + 2 <= slot->size(3), "slot range");
    sp = bf16m(*slot) + slot_off;
    ss = (int)slot->size(3);
  }
  c10::DeviceGuard gd(flow.device());
  launch_flow_prep(flow.data_ptr<float>(), bf16m(flowb), sp, ss, (int)B, (int)(H * W), cur_stream());
}

// AdamW over lists of fp32 tensors with the global-norm gradient clip folded in (adamw.hip);
// returns the device pair [clip coefficient, total gradient norm]
// One AdamW step over every parameter group (global-norm clip over all of them), with the fp16
// GradScaler folded in: inv_scale (1/S, device) unscales the gradients inside the kernels, and an
// overflow (non-finite norm) skips the whole step on the device and sets found_inf.  Per group g:
// lr_t[g] (a one-element fp32 device tensor, or an empty tensor for the host value lr[g]),
// beta1/beta2/eps/wd[g]; per tensor: its group index and its device step counter (fp32, 1 elem).
// Returns (gradient multiplier, total unscaled norm, found_inf) as a 3-element device tensor.
Tensor adamw_step_(const std::vector<Tensor>& params, const std::vector<Tensor>& grads,
                   const std::vector<Tensor>& exp_avg, const std::vector<Tensor>& exp_avg_sq,
                   const std::vector<Tensor>& steps, const std::vector<int64_t>& group_of,
                   const std::vector<Tensor>& lr_t, const std::vector<double>& lr,
                   const std::vector<double>& beta1, const std::vector<double>& beta2,
                   const std::vector<double>& eps, const std::vector<double>& wd, double max_norm,
                   const c10::optional<Tensor>& inv_scale, const c10::optional<Tensor>& found_inf,
                   bool write_grad) {
  const size_t T = params.size();
  TORCH_CHECK(T > 0 && grads.size() == T && exp_avg.size() == T && exp_avg_sq.size() == T &&
                  steps.size() == T && group_of.size() == T,
              "adamw: tensor lists must have the same length");
  const size_t G = lr.size();
  TORCH_CHECK(G >= 1 && lr_t.size() == G && beta1.size() == G && beta2.size() == G &&
                  eps.size() == G && wd.size() == G,
              "adamw: per-group hyper-parameter lists must have the same length");
  const auto dev = params[0].device();
  // same flat walk: equal sizes and equal strides over the dims of size > 1 (a size-1 dim's stride
  // does not move the walk: a channels_last 1x1 conv weight and its contiguous gradient agree)
  auto same_walk = [](const Tensor& x, const Tensor& y) {
    if (x.sizes() != y.sizes()) return false;
    for (int64_t d = 0; d < x.dim(); ++d)
      if (x.size(d) > 1 && x.stride(d) != y.stride(d)) return false;
    return true;
  };
  for (size_t i = 0; i < T; ++i) {
    for (const Tensor* t : {&params[i], &grads[i], &exp_avg[i], &exp_avg_sq[i]}) {
      // the kernels walk the four tensors as flat arrays: any dense layout, the same for all four
      // (a channels_last model's weights, their gradients and moments)
      TORCH_CHECK(t->is_cuda() && t->device() == dev && t->scalar_type() == at::kFloat &&
                      t->is_non_overlapping_and_dense() && same_walk(*t, params[i]) &&
                      t->numel() == params[i].numel(),
                  "adamw: dense fp32 tensors of one size and layout on one GPU");
    }
    TORCH_CHECK(steps[i].is_cuda() && steps[i].device() == dev && steps[i].scalar_type() == at::kFloat &&
                    steps[i].numel() == 1,
                "adamw: step counters must be one-element fp32 tensors on the parameters' GPU");
    TORCH_CHECK(group_of[i] >= 0 && group_of[i] < (int64_t)G, "adamw: group index out of range");
  }
  auto dev_scalar = [&](const c10::optional<Tensor>& t, const char* name) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->device() == dev && t->scalar_type() == at::kFloat && t->numel() == 1,
                "adamw: ", name, " must be a one-element fp32 tensor on the parameters' GPU");
    return t->data_ptr<float>();
  };
  const float* isp = dev_scalar(inv_scale, "inv_scale");
  float* fip = dev_scalar(found_inf, "found_inf");
  const int64_t CH = adam_chunk_elems();
  const int64_t tab_bytes = (int64_t)T * (int64_t)sizeof(AdamTensor);
  const int64_t grp_off = (tab_bytes + (int64_t)(T + 1) * 4 + 15) / 16 * 16;
  const int64_t grp_bytes = (int64_t)G * (int64_t)sizeof(AdamGroup);
  Tensor host = at::empty({grp_off + grp_bytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  uint8_t* hb = host.data_ptr<uint8_t>();
  AdamTensor* ht = reinterpret_cast<AdamTensor*>(hb);
  int* hc = reinterpret_cast<int*>(hb + tab_bytes);
  AdamGroup* hg = reinterpret_cast<AdamGroup*>(hb + grp_off);
  hc[0] = 0;
  for (size_t i = 0; i < T; ++i) {
    ht[i] = AdamTensor{params[i].data_ptr<float>(), grads[i].data_ptr<float>(),
                       exp_avg[i].data_ptr<float>(), exp_avg_sq[i].data_ptr<float>(),
                       params[i].numel(), steps[i].data_ptr<float>(), (int)group_of[i]};
    const int64_t nc = (params[i].numel() + CH - 1) / CH;
    TORCH_CHECK((int64_t)hc[i] + nc < (int64_t(1) << 30), "adamw: too many chunks");
    hc[i + 1] = hc[i] + (int)nc;
  }
  for (size_t g = 0; g < G; ++g) {
    const float* lp = nullptr;
    if (lr_t[g].defined() && lr_t[g].numel() > 0) {
      TORCH_CHECK(lr_t[g].is_cuda() && lr_t[g].device() == dev && lr_t[g].scalar_type() == at::kFloat &&
                      lr_t[g].numel() == 1,
                  "adamw: lr tensor must be a one-element fp32 tensor on the parameters' GPU");
      lp = lr_t[g].data_ptr<float>();
    }
    // 1 - beta in double, like torch (1 - 0.999 from a float-rounded beta is 1.3e-5 off)
    hg[g] = AdamGroup{lp, (float)lr[g], (float)wd[g], (float)beta1[g], (float)beta2[g],
                      (float)(1.0 - beta1[g]), (float)(1.0 - beta2[g]), (float)eps[g]};
  }
  const int nchunks = hc[T];
  c10::DeviceGuard g(dev);
  // pinned source + stream-ordered copy: no host sync (the caching host allocator keeps the
  // block until the copy has run)
  Tensor dtab = host.to(dev, /*non_blocking=*/true);
  Tensor out = at::empty({(int64_t)nchunks + 3}, params[0].options());
  uint8_t* db = dtab.data_ptr<uint8_t>();
  const bool need_norm = max_norm > 0.0 || isp != nullptr;
  launch_adamw_multi(reinterpret_cast<const AdamTensor*>(db), reinterpret_cast<const int*>(db + tab_bytes),
                     (int)T, nchunks, reinterpret_cast<const AdamGroup*>(db + grp_off), (float)max_norm,
                     isp, need_norm ? 1 : 0, write_grad ? 1 : 0, out.data_ptr<float>(),
                     out.data_ptr<float>() + nchunks, fip, cur_stream());
  return out.narrow(0, nchunks, 3);
}

// dcorr level 0 (B, N, N) straight from the iterations' bf16 lookup-output gradients
Tensor corr_tap_reduce(const std::vector<Tensor>& coords, const std::vector<Tensor>& douts,
                       int64_t H, int64_t W, int64_t levels, int64_t radius, double inv_sqrt_c,
                       bool out_bf16, int64_t pitch_mult, bool split, bool split_out) {
  // split fp32 tap gradients ([hi | lo] bf16 halves): the fold is linear in the taps, so each
  // iteration enters twice -- its hi and its lo half -- with the same coordinates
  const size_t rep = split ? 2 : 1;
  TORCH_CHECK(!coords.empty() && coords.size() == douts.size() && rep * coords.size() <= RAFT_MAX_WIN,
              "1..", RAFT_MAX_WIN / rep, " iterations");
  TORCH_CHECK(radius == 3 || radius == 4, "radius must be 3 or 4");
  TORCH_CHECK(levels >= 1 && levels <= 4, "1..4 levels");
  const int64_t B = coords[0].size(0), N = H * W;
  const int64_t D = 2 * radius + 1;
  const int64_t cbuf = douts[0].size(-1);
  const int64_t cuse = split ? cbuf / 2 : cbuf;
  TORCH_CHECK(!split || (cbuf % 16 == 0 && douts[0].scalar_type() == at::kBFloat16), "split taps: bf16 halves");
  TapList tl{};
  for (size_t k = 0; k < coords.size(); ++k) {
    check_cuda_f32(coords[k], "coords");
    TORCH_CHECK(coords[k].dim() == 4 && coords[k].size(0) == B && coords[k].size(1) == 2 &&
                    coords[k].size(2) == H && coords[k].size(3) == W,
                "coords shape");
    check_nhwc(douts[k], B, H, W, "tap gradient", douts[0].scalar_type());
    TORCH_CHECK(douts[k].scalar_type() == at::kBFloat16 || douts[k].scalar_type() == at::kHalf,
                "tap gradients must be bf16 or fp16");
    TORCH_CHECK(douts[k].size(3) == cbuf && cbuf % 8 == 0 && cuse >= levels * D * D,
                "tap gradient rows must share a width >= levels*(2r+1)^2, multiple of 8");
    for (size_t h = 0; h < rep; ++h) {
      tl.coords[rep * k + h] = coords[k].data_ptr<float>();
      tl.dout[rep * k + h] = u16(douts[k]) + h * cuse;
    }
  }
  tl.n = (int)(rep * coords.size());
  tl.cbuf = (int)cbuf;
  tl.tf16 = douts[0].scalar_type() == at::kHalf ? 1 : 0;
  // row pitch: N, or N rounded up to pitch_mult (zero columns: the MFMA backward GEMMs' K padding)
  TORCH_CHECK(pitch_mult >= 0 && pitch_mult % 2 == 0, "pitch_mult must be even");
  const int64_t ldo = pitch_mult > 0 ? (N + pitch_mult - 1) / pitch_mult * pitch_mult : N;
  tl.ldo = (int)ldo;
  const int lds = corr_tap_reduce_lds_bytes((int)H, (int)W, (int)levels, (int)radius);
  TORCH_CHECK(lds <= 64 * 1024, "feature map too large for the LDS plane reduction");
  c10::DeviceGuard g(coords[0].device());
  // split_out: the fp32 dC as its split-bf16 planes [hi | lo] (2, B, N, ldo) -- the operand of
  // the split MFMA backward GEMMs (corr_bwd_fmaps_split)
  Tensor out = split_out ? at::empty({2, B, N, ldo}, coords[0].options().dtype(at::kBFloat16))
                         : at::empty({B, N, ldo}, coords[0].options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  // overflow list of the union-box fold (count + pixel indices)
  Tensor list = at::empty({1 + B * N}, coords[0].options().dtype(at::kInt));
  TORCH_CHECK(launch_corr_tap_reduce(tl, (int)levels, (int)B, (int)H, (int)W, (int)radius,
                                     (float)inv_sqrt_c, out.data_ptr(), split_out ? 2 : (out_bf16 ? 1 : 0),
                                     list.data_ptr<int>(), cur_stream()),
              "unsupported radius / levels");
  return out;
}

// feature-map gradients of the all-pairs correlation: dc (B, N, ldc) bf16 from corr_tap_reduce
// with pitch_mult 64, f1 / f2 (B, H, W, C) bf16 -> [dF1 = dC F2, dF2 = dC^T F1] as (B, H, W, C)
std::vector<Tensor> corr_bwd_fmaps(const Tensor& dc, const Tensor& f1, const Tensor& f2) {
  TORCH_CHECK(f1.dim() == 4 && f1.sizes() == f2.sizes(), "fmaps must be (B, H, W, C) of one shape");
  const int64_t B = f1.size(0), H = f1.size(1), W = f1.size(2), C = f1.size(3), N = H * W;
  check_nhwc(f1, B, H, W, "fmap1", at::kBFloat16);
  check_nhwc(f2, B, H, W, "fmap2", at::kBFloat16);
  TORCH_CHECK(dc.is_cuda() && dc.is_contiguous() && dc.scalar_type() == at::kBFloat16 && dc.dim() == 3 &&
                  dc.size(0) == B && dc.size(1) == N && dc.size(2) >= N && dc.size(2) % 64 == 0,
              "dcorr must be a contiguous bf16 (B, N, ldc) tensor, ldc a multiple of 64 >= N");
  TORCH_CHECK(C % 128 == 0, "channels must be a multiple of 128");
  const int64_t ldc = dc.size(2);
  TORCH_CHECK(N * ldc * 2 < (int64_t(1) << 31) && C * ldc * 2 < (int64_t(1) << 31) &&
                  N * C * 2 < (int64_t(1) << 31),
              "per-image operands exceed the 2 GiB buffer-descriptor range");
  c10::DeviceGuard g(dc.device());
  Tensor f2t = at::empty({B, C, ldc}, dc.options());
  Tensor g1 = at::empty({B, H, W, C}, dc.options());
  Tensor g2 = at::empty({B, H, W, C}, dc.options());
  TORCH_CHECK(launch_corr_bwd_fmaps(bf16p(dc), (int)ldc, bf16p(f1), bf16p(f2), bf16m(f2t), bf16m(g1),
                                    bf16m(g2), (int)B, (int)N, (int)C, cur_stream()),
              "corr backward GEMM launch");
  return {g1, g2};
}

// fp32 correlation (fp16 / fp32 schedules): dc2 (2, B, N, ldc) bf16 split planes from
// corr_tap_reduce(split_out=True, pitch_mult=64), f1 / f2 fp32 (B, C, H, W) contiguous ->
// [dF1 = dC F2, dF2 = dC^T F1] fp32 (B, H, W, C), three split-bf16 MFMA passes per GEMM
std::vector<Tensor> corr_bwd_fmaps_split(const Tensor& dc2, const Tensor& f1, const Tensor& f2) {
  TORCH_CHECK(f1.dim() == 4 && f1.sizes() == f2.sizes(), "fmaps must be (B, C, H, W) of one shape");
  const int64_t B = f1.size(0), C = f1.size(1), H = f1.size(2), W = f1.size(3), N = H * W;
  for (const Tensor* t : {&f1, &f2}) {
    check_cuda_f32(*t, "fmap");
    TORCH_CHECK(t->is_contiguous(), "fmaps must be contiguous NCHW fp32");
  }
  TORCH_CHECK(dc2.is_cuda() && dc2.is_contiguous() && dc2.scalar_type() == at::kBFloat16 && dc2.dim() == 4 &&
                  dc2.size(0) == 2 && dc2.size(1) == B && dc2.size(2) == N && dc2.size(3) >= N &&
                  dc2.size(3) % 64 == 0,
              "dcorr must be the contiguous split planes (2, B, N, ldc) bf16, ldc a multiple of 64 >= N");
  TORCH_CHECK(C % 128 == 0, "channels must be a multiple of 128");
  const int64_t ldc = dc2.size(3);
  TORCH_CHECK(N * ldc * 2 < (int64_t(1) << 31) && C * ldc * 2 < (int64_t(1) << 31) &&
                  N * C * 2 < (int64_t(1) << 31),
              "per-image operands exceed the 2 GiB buffer-descriptor range");
  c10::DeviceGuard g(dc2.device());
  Tensor f2s = at::empty({2, B, C, ldc}, dc2.options());
  Tensor f1s = at::empty({2, B, N, C}, dc2.options());
  Tensor g1 = at::empty({B, H, W, C}, f1.options());
  Tensor g2 = at::empty({B, H, W, C}, f1.options());
  TORCH_CHECK(launch_corr_bwd_fmaps_split(bf16p(dc2), (int)ldc, f1.data_ptr<float>(), f2.data_ptr<float>(),
                                          bf16m(f2s), bf16m(f1s), g1.data_ptr<float>(), g2.data_ptr<float>(),
                                          (int)B, (int)N, (int)C, cur_stream()),
              "split corr backward GEMM launch");
  return {g1, g2};
}

// ------------------------------------------------------------------ flow_head.conv2 (256 -> 2)
// Weights arrive as bf16 pair tables built by the update block's packing gather:
// wf = W[o][c][t] as [t][o][c] (2304 bf16), wd = W[o][c][t] as [t][c][o] (4608 bf16).
const uint32_t* fh2_pairs(const Tensor& t, int64_t n, const char* name, at::ScalarType st) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == st, name,
              " must be a contiguous GPU tensor of the activation dtype");
  TORCH_CHECK(t.numel() == n, name, " must hold ", n, " elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-B aligned");
  return reinterpret_cast<const uint32_t*>(t.data_ptr());
}

// out (B,2,H,W) fp32 = conv3x3(in[..., 0:256]) + bias
// coords (optional): cnew = coords + out, fnew = cnew - coords_grid (the iteration's coordinate
// update, `core/raft.py:134-135`, in the same launch)
void fh2_fwd_(const Tensor& in, const Tensor& wf, const Tensor& b, const Tensor& out,
              const c10::optional<Tensor>& coords, const c10::optional<Tensor>& cnew,
              const c10::optional<Tensor>& fnew) {
  TORCH_CHECK(in.dim() == 4, "in must be (B,H,W,C)");
  const int64_t B = in.size(0), H = in.size(1), W = in.size(2), cs = in.size(3);
  const at::ScalarType st = op16(in);
  check_nhwc(in, B, H, W, "fh2 in", st);
  const uint32_t* wp = fh2_pairs(wf, 9 * 2 * 256, "fh2 wf", st);
  check_cuda_f32(b, "fh2 bias");
  TORCH_CHECK(b.numel() == 2, "fh2 bias must have 2 elements");
  check_cuda_f32(out, "fh2 out");
  TORCH_CHECK(out.dim() == 4 && out.size(0) == B && out.size(1) == 2 && out.size(2) == H &&
              out.size(3) == W, "fh2 out must be (B,2,H,W)");
  const bool upd = coords.has_value() && coords->defined();
  if (upd) {
    TORCH_CHECK(cnew.has_value() && fnew.has_value(), "fh2_fwd: coords needs cnew and fnew");
    for (const Tensor* t : {&*coords, &*cnew, &*fnew}) {
      check_cuda_f32(*t, "fh2 coords");
      TORCH_CHECK(t->sizes() == out.sizes() && t->is_contiguous(), "fh2 coords must be (B,2,H,W)");
    }
  }
  c10::DeviceGuard gd(in.device());
  TORCH_CHECK(launch_fh2_fwd(u16(in), (int)cs, wp, b.data_ptr<float>(), out.data_ptr<float>(),
                             (int)B, (int)H, (int)W, st == at::kHalf, cur_stream(),
                             upd ? coords->data_ptr<float>() : nullptr,
                             upd ? cnew->data_ptr<float>() : nullptr,
                             upd ? fnew->data_ptr<float>() : nullptr),
              "fh2_fwd: input needs >= 256 channels, a multiple of 8");
}

// dx[..., 0:256] (bf16) = [fm[..., 0:256] > 0] * conv3x3^T(gout)
void fh2_dgrad_(const Tensor& gout, const Tensor& wd, const Tensor& fm, const Tensor& dx) {
  check_cuda_f32(gout, "fh2 gout");
  TORCH_CHECK(gout.dim() == 4 && gout.size(1) == 2, "gout must be (B,2,H,W)");
  const int64_t B = gout.size(0), H = gout.size(2), W = gout.size(3);
  const at::ScalarType st = op16(fm);
  check_nhwc(fm, B, H, W, "fh2 fm", st);
  check_nhwc(dx, B, H, W, "fh2 dx", st);
  const uint32_t* wp = fh2_pairs(wd, 9 * 256 * 2, "fh2 wd", st);
  c10::DeviceGuard gd(gout.device());
  TORCH_CHECK(launch_fh2_dgrad(gout.data_ptr<float>(), wp, u16(fm), (int)fm.size(3), u16m(dx),
                               (int)dx.size(3), (int)B, (int)H, (int)W, st == at::kHalf, cur_stream()),
              "fh2_dgrad: fm / dx need >= 256 channels, multiples of 8");
}

// part (G, 2*2304 + 2) fp32 <- per-workgroup partial [dw (o, t*256 + c) | db] sums over all items
void fh2_wgrad_(const std::vector<Tensor>& gouts, const std::vector<Tensor>& ins, const Tensor& part) {
  const int64_t n = (int64_t)gouts.size();
  TORCH_CHECK(n >= 1 && n <= RAFT_FH2_MAX_ITEMS && (int64_t)ins.size() == n, "1..",
              RAFT_FH2_MAX_ITEMS, " (gout, in) items");
  const int64_t B = gouts[0].size(0), H = gouts[0].size(2), W = gouts[0].size(3);
  const int64_t cs = ins[0].size(3);
  Fh2Items it{};
  it.n = (int)n;
  const at::ScalarType st = op16(ins[0]);
  for (int64_t i = 0; i < n; ++i) {
    check_cuda_f32(gouts[i], "fh2 gout");
    TORCH_CHECK(gouts[i].dim() == 4 && gouts[i].size(0) == B && gouts[i].size(1) == 2 &&
                gouts[i].size(2) == H && gouts[i].size(3) == W, "all gouts must be (B,2,H,W)");
    check_nhwc(ins[i], B, H, W, "fh2 wgrad input", st);
    TORCH_CHECK(ins[i].size(3) == cs, "all items' inputs must share a layout");
    it.gout[i] = gouts[i].data_ptr<float>();
    it.in[i] = u16(ins[i]);
  }
  check_cuda_f32(part, "fh2 part");
  TORCH_CHECK(part.dim() == 2 && part.size(1) == 2 * 9 * 256 + 2, "fh2 part must be (G, 4610)");
  // rows beyond the number of (item, image, 8-row) units are written as zeros
  TORCH_CHECK(part.size(0) >= 1 && part.size(0) <= 65535, "fh2 part needs 1..65535 rows");
  c10::DeviceGuard gd(part.device());
  TORCH_CHECK(launch_fh2_wgrad(it, (int)cs, (int)B, (int)H, (int)W, part.data_ptr<float>(),
                               (int)part.size(0), st == at::kHalf, cur_stream()),
              "fh2_wgrad: inputs need >= 256 channels, a multiple of 8");
}

// patch (B,H,W,128) bf16 = 7x7 neighbourhood of the flow (tap-major, 2 ch; 98..127 zero);
// optionally slot[..., off:off+2] = flow
void f1_patch_(const Tensor& flow, const Tensor& patch, const c10::optional<Tensor>& slot,
               int64_t slot_off) {
  check_cuda_f32(flow, "flow");
  TORCH_CHECK(flow.dim() == 4 && flow.size(1) == 2, "flow must be (B,2,H,W)");
  const int64_t B = flow.size(0), H = flow.size(2), W = flow.size(3);
  const at::ScalarType st = op16(patch);
  check_nhwc(patch, B, H, W, "patch", st);
  // 256 channels: split fp32 [hi (128) | lo (128)] (the fp32 schedule); the slot likewise
  TORCH_CHECK(patch.size(3) == 128 || (patch.size(3) == 256 && st == at::kBFloat16),
              "patch must have 128 channels (256: split fp32 pairs)");
  const bool spl = patch.size(3) == 256;
  uint16_t* sp = nullptr;
  int ss = 0;
  if (slot.has_value() && slot->defined()) {
    check_nhwc(*slot, B, H, W, "slot", st);
    TORCH_CHECK(slot_off >= 0 && slot_off + 2 <= (spl ? slot->size(3) / 2 : slot->size(3)), "slot range");
    TORCH_CHECK(!spl || slot->size(3) % 2 == 0, "split slot: two halves");
    sp = u16m(*slot) + slot_off;
    ss = (int)slot->size(3);
  }
  c10::DeviceGuard gd(flow.device());
  launch_f1_patch(flow.data_ptr<float>(), u16m(patch), sp, ss, (int)B, (int)H, (int)W,
                  spl ? 2 : (st == at::kHalf ? 1 : 0), cur_stream());
}

}  // namespace

TORCH_LIBRARY(raft_amd, m) {
  m.def("corr_build(Tensor f1, Tensor f2, int levels) -> Tensor[]");
  m.def("corr_lookup_fwd(Tensor[] pyr, Tensor coords, int radius) -> Tensor");
  m.def("corr_lookup_bwd_(Tensor(a!)[] gpyr, Tensor coords, Tensor dout, int radius) -> ()");
  m.def("corr_pyr_grad_reduce(Tensor[] gpyr, float inv_sqrt_c) -> Tensor");
  m.def("corr_otf_fwd_(Tensor f1, Tensor[] f2, Tensor coords, int radius, Tensor(a!) out, Tensor[] lo) -> ()");
  m.def("corr_otf_bwd_(Tensor f1, Tensor[] f2, Tensor coords, Tensor dout, Tensor(a!) df1, Tensor(b!)[] df2, int radius, int dslo=0) -> ()");
  m.def("conv_tune_table() -> int[]", &conv_tune_table);
  m.def("conv_set_forced_cfg(int idx) -> ()", [](int64_t idx) { conv_set_forced_cfg((int)idx); });
  m.def("conv_set_autotune(int mode) -> ()", [](int64_t mode) { conv_set_autotune((int)mode); });
  m.def("conv_autotune_runs() -> int", []() -> int64_t { return conv_autotune_runs(); });
  m.def("phase_mark() -> ()", []() { launch_phase_marker(cur_stream()); });
  m.def("conv_tune_import(int[] rows) -> int", [](std::vector<int64_t> rows) -> int64_t {
    TORCH_CHECK(rows.size() % 13 == 0, "tuned table rows have 13 entries");
    std::vector<int> r(rows.begin(), rows.end());
    return conv_import_tuned(r.data(), (int)(r.size() / 13));
  });
  m.def("norm_fwd_(Tensor x, int mode, int relu, Tensor? gamma, Tensor? beta, Tensor? cbias, Tensor(a!)? rmean, Tensor(b!)? rvar, float momentum, float eps, Tensor? res, Tensor(c!) y, Tensor(d!)? ysplit=None, Tensor? tstats=None, int tiles=0) -> Tensor[]");
  m.def("norm_bwd_(Tensor dy, Tensor x, Tensor? y, Tensor mean, Tensor invstd, int mode, int relu, Tensor? gamma, Tensor? beta, Tensor(a!)? dgamma, Tensor(b!)? dbeta, Tensor(c!)? dcbias, Tensor(d!) dx, Tensor? dy2=None, Tensor? yres=None, Tensor(e!)? gout=None, Tensor(f!)? dxsplit=None) -> ()");
  m.def("add_relu_(Tensor a, Tensor b, Tensor(a!) out) -> ()");
  m.def("relu_mask_(Tensor dy, Tensor y, Tensor(a!) g, Tensor? dy2=None) -> ()");
  m.def("gather_cast_(Tensor[] srcs, Tensor idx, Tensor(a!) out, int lo_from=-1) -> ()");
  m.def("image_prep_(Tensor a, Tensor b, Tensor(a!) out) -> ()");
  m.def("ctx_act_(Tensor cnet, int hdim, Tensor(a!) h, Tensor(b!) x) -> ()");
  m.def("ctx_act_bwd_(Tensor? gh, Tensor? gx, Tensor h, Tensor x, Tensor(a!) gin) -> ()");
  m.def("corr_otf_window_bwd_(Tensor f1, Tensor[] f2, Tensor[] coords, Tensor[] douts, Tensor(a!) df1, Tensor(b!)[] df2, int radius) -> ()");
  m.def("corr_build_bf16(Tensor f1, Tensor f2, int levels, bool pyr_bf16=False) -> Tensor[]");
  m.def("conv_wgrad_taps_(Tensor[] gs, int g_off, Tensor[] ins, int[] in_off, int[] in_cnt, int kh, "
        "int kw, int ph, int pw, int cout, Tensor dw, Tensor? db, int splits=0, bool split=False) -> ()");
  m.def("convex_up_fwd(Tensor flow, Tensor mask, bool nhwc=False) -> Tensor");
  m.def("convex_up_bwd(Tensor flow, Tensor mask, Tensor dout, bool nhwc=False) -> Tensor[]");
  m.def("corr_lookup_nhwc_(Tensor[] pyr, Tensor coords, int radius, Tensor(a!) out, bool split=False) -> ()");
  m.def("corr_window_grad(Tensor coords, Tensor dout, int levels, int radius) -> Tensor");
  m.def("corr_window_reduce(Tensor[] coords, Tensor[] wgs, int H, int W, int levels, int radius, float inv_sqrt_c, bool out_bf16=False) -> Tensor");
  m.def("conv_dgrad_(Tensor[] ins, int[] in_off, int[] in_cnt, Tensor wpk, int kh, int kw, int ph, int pw, int cin_small, float scale, Tensor(a!)[] outs, int[] out_off, int[] out_cnt, int[] out_real, int[] out_acc, Tensor[] relu_y, int[] relu_off, int[] gate_mode, Tensor[] gate_t, int[] out_kcin=[], bool split=False) -> ()");
  m.def("split_hilo_(Tensor x, Tensor(a!) out) -> ()");
  m.def("conv_enc64_(Tensor x, Tensor wpk, Tensor(a!) out, Tensor(b!)? part=None) -> ()");
  m.def("stem_conv_fwd_(Tensor x, Tensor w, Tensor(a!) out) -> ()");
  m.def("stem_conv_wgrad(Tensor x, Tensor gy) -> Tensor");
  m.def("relu_bwd_(Tensor g, int g_off, Tensor? y, int y_off, Tensor(a!) out, int o_off, int C, float scale, bool split=False) -> ()");
  m.def("gru_q_bwd_(Tensor dh, Tensor z, Tensor q, Tensor hprev, Tensor(a!) dpre_q, Tensor(b!) dz, Tensor(c!) dhprev) -> ()");
  m.def("gru_zr_bwd_(Tensor drh, Tensor dz, Tensor z, Tensor r, Tensor hprev, Tensor(a!) dpre_zr, Tensor(b!) dhprev) -> ()");
  m.def("sum_bf16_(Tensor[] ins, Tensor? carry, Tensor(a!) out) -> ()");
  m.def("flow_prep_(Tensor flow, Tensor(a!) flowb, Tensor(b!)? slot, int slot_off) -> ()");
  m.def("seq_loss_fwd(Tensor[] preds, Tensor gt, Tensor valid, float gamma, float max_flow) -> Tensor");
  m.def("seq_loss_bwd(Tensor[] preds, Tensor gt, Tensor valid, Tensor dloss, float gamma, float max_flow) -> Tensor[]");
  m.def("warp_fwd(Tensor img, Tensor flow, float sx, float bx, float sy, float by) -> Tensor");
  m.def("warp_bwd(Tensor img, Tensor flow, Tensor dout, float sx, float bx, float sy, float by) -> Tensor[]");
  m.def("conv_fwd_(Tensor[] ins, int[] in_off, int[] in_cnt, Tensor wpk, Tensor? bias, int kh, int kw, int ph, int pw, int cout, int cin_small, int epi, int bn, float scale, int split, Tensor(a!)[] outs, int[] out_off, Tensor[] aux, int[] aux_off) -> ()");
  m.def("conv_wgrad_multi_(Tensor[] gs, int g_off, Tensor[] ins, int[] in_off, int[] in_cnt, int kh, int kw, int ph, int pw, int cout, Tensor(a!) dw, Tensor(b!)? db, int pix_per_split) -> ()");
  m.def("f1_patch_(Tensor flow, Tensor(a!) patch, Tensor(b!)? slot, int slot_off) -> ()");
  m.def("adamw_step_(Tensor(a!)[] params, Tensor(b!)[] grads, Tensor(c!)[] exp_avg, Tensor(d!)[] exp_avg_sq, Tensor(e!)[] steps, int[] group_of, Tensor[] lr_t, float[] lr, float[] beta1, float[] beta2, float[] eps, float[] wd, float max_norm, Tensor? inv_scale=None, Tensor(f!)? found_inf=None, bool write_grad=False) -> Tensor");
  m.def("corr_tap_reduce(Tensor[] coords, Tensor[] douts, int H, int W, int levels, int radius, float inv_sqrt_c, bool out_bf16, int pitch_mult=0, bool split=False, bool split_out=False) -> Tensor");
  m.def("corr_bwd_fmaps(Tensor dc, Tensor f1, Tensor f2) -> Tensor[]");
  m.def("corr_bwd_fmaps_split(Tensor dc2, Tensor f1, Tensor f2) -> Tensor[]");
  m.def("fh2_fwd_(Tensor inp, Tensor wf, Tensor b, Tensor(a!) out, Tensor? coords=None, "
        "Tensor(b!)? cnew=None, Tensor(c!)? fnew=None) -> ()");
  m.def("fh2_dgrad_(Tensor gout, Tensor wd, Tensor fm, Tensor(a!) dx) -> ()");
  m.def("fh2_wgrad_(Tensor[] gouts, Tensor[] ins, Tensor(a!) part) -> ()");
  m.def("conv_wgrad_(Tensor g, int g_off, Tensor[] ins, int[] in_off, int[] in_cnt, int kh, int kw, int ph, int pw, int cout, int cin_small, Tensor(a!) dw, Tensor(b!)? db, int pix_per_split) -> ()");
}

TORCH_LIBRARY_IMPL(raft_amd, CUDA, m) {
  m.impl("corr_build", &corr_build);
  m.impl("corr_lookup_fwd", &corr_lookup_fwd);
  m.impl("corr_lookup_bwd_", &corr_lookup_bwd_);
  m.impl("corr_pyr_grad_reduce", &corr_pyr_grad_reduce);
  m.impl("corr_otf_fwd_", &corr_otf_fwd_);
  m.impl("corr_otf_bwd_", &corr_otf_bwd_);
  m.impl("corr_otf_window_bwd_", &corr_otf_window_bwd_);
  m.impl("norm_fwd_", &norm_fwd_);
  m.impl("norm_bwd_", &norm_bwd_);
  m.impl("f1_patch_", &f1_patch_);
  m.impl("adamw_step_", &adamw_step_);
  m.impl("corr_tap_reduce", &corr_tap_reduce);
  m.impl("corr_bwd_fmaps", &corr_bwd_fmaps);
  m.impl("corr_bwd_fmaps_split", &corr_bwd_fmaps_split);
  m.impl("fh2_fwd_", &fh2_fwd_);
  m.impl("fh2_dgrad_", &fh2_dgrad_);
  m.impl("fh2_wgrad_", &fh2_wgrad_);
  m.impl("add_relu_", &add_relu_);
  m.impl("relu_mask_", &relu_mask_);
  m.impl("gather_cast_", &gather_cast_);
  m.impl("image_prep_", &image_prep_);
  m.impl("ctx_act_", &ctx_act_);
  m.impl("ctx_act_bwd_", &ctx_act_bwd_);
  m.impl("corr_build_bf16", &corr_build_bf16);
  m.impl("conv_wgrad_taps_", &conv_wgrad_taps_);
  m.impl("convex_up_fwd", &convex_up_fwd);
  m.impl("convex_up_bwd", &convex_up_bwd);
  m.impl("seq_loss_fwd", &seq_loss_fwd);
  m.impl("seq_loss_bwd", &seq_loss_bwd);
  m.impl("warp_fwd", &warp_fwd);
  m.impl("warp_bwd", &warp_bwd);
  m.impl("conv_fwd_", &conv_fwd_);
  m.impl("conv_wgrad_", &conv_wgrad_);
  m.impl("conv_wgrad_multi_", &conv_wgrad_multi_);
  m.impl("corr_lookup_nhwc_", &corr_lookup_nhwc_);
  m.impl("corr_window_grad", &corr_window_grad);
  m.impl("corr_window_reduce", &corr_window_reduce);
  m.impl("conv_dgrad_", &conv_dgrad_);
  m.impl("relu_bwd_", &relu_bwd_);
  m.impl("split_hilo_", &split_hilo_);
  m.impl("conv_enc64_", &conv_enc64_);
  m.impl("stem_conv_fwd_", &stem_conv_fwd_);
  m.impl("stem_conv_wgrad", &stem_conv_wgrad);
  m.impl("gru_q_bwd_", &gru_q_bwd_);
  m.impl("gru_zr_bwd_", &gru_zr_bwd_);
  m.impl("flow_prep_", &flow_prep_);
  m.impl("sum_bf16_", &sum_bf16_);
}
