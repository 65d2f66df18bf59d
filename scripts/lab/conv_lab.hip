// Stand-alone timing lab for the update-block conv kernels (no torch): a 1x5 ConvGRU conv at the
// chairs training shape (B=12, 46x62, [h | mf] = 2 x 128 channels -> 256) through the library's
// LDS-DMA kernel and instrumented copies of it.  Build + run (GPU box):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I pytorch_raft_amd/csrc/kernels \
//         scripts/lab/conv_lab.hip -o /tmp/conv_lab && /tmp/conv_lab
#include "conv_glds.hip"
#include "conv_v3.h"
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <algorithm>

using namespace conv_detail;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// ---------------------------------------------------------------- instrumented kernel
// conv_fwd_glds_kernel with s_memtime stamps (wave 0 lane 0 of every workgroup):
// [0] entry, [1] first K step's data landed, [2] main loop done, [3] epilogue done, [4] XCC id
template <int TM, int TN, int WVM, int EPI, int NS, int OCCV>
__global__ __launch_bounds__(NT, OCCV) void conv_stamp_kernel(ConvFwdArgs a, unsigned long long* st) {
  using T = ConvTile<TM, TN, WVM>;
  constexpr int BM = T::BM, BN = T::BN, WM = 32 * TM, WN = 32 * TN;
  constexpr int WAVES_N = T::WVN;
  constexpr int A_CHUNKS = BM * 8, B_CHUNKS = BN * 8;
  constexpr int A_PER = A_CHUNKS / NT, B_PER = B_CHUNKS / NT;
  constexpr int STAGE = A_CHUNKS + B_CHUNKS;
  constexpr int LPS = A_PER + B_PER;
  __shared__ __attribute__((aligned(16))) uint4 smem[NS * STAGE];
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0, t2 = 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  int mt, nt;
  if (!conv_tile_coords(raft_cdiv(P, BM), raft_cdiv(a.cout, BN), mt, nt)) return;
  const int m0 = mt * BM, n0 = nt * BN;
  int a_pix[A_PER], a_y[A_PER], a_x[A_PER], a_lc[A_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e >> 3;
    const int m = m0 + row;
    const int mm = m < P ? m : 0;
    const int r = mm % HW;
    a_pix[j] = mm;
    a_y[j] = m < P ? r / a.W : -(1 << 20);
    a_x[j] = r % a.W;
    a_lc[j] = ((e & 7) ^ ((row >> 1) & 7)) * 8;
  }
  uint32_t b_off[B_PER];
#pragma unroll
  for (int j = 0; j < B_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e >> 3;
    const int n = n0 + row;
    const int lc = (e & 7) ^ ((row >> 1) & 7);
    b_off[j] = n < a.cout ? (uint32_t)(((int64_t)n * a.kpad + lc * 8) * 2) : OOB;
  }
  const int nchunk = a.cin_pad / BK;
  const int ntap = a.KH * a.KW;
  const int steps = ntap * nchunk;
  rsrc_t seg_rs[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int qq = q < a.nseg ? q : 0;
    seg_rs[q] = make_rsrc(a.seg[qq].ptr, (uint32_t)P * a.seg[qq].stride * 2u);
  }
  const rsrc_t w_rs = make_rsrc(a.wpk, (uint32_t)a.cout * a.kpad * 2u);
  const uint32_t lds0 = raft_lds_addr(smem) + __builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int t, int buf) {
    const int ch = t / ntap, tap = t - ch * ntap;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const int c0 = ch * BK;
    int s = 0, sbase = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (s + 1 < a.nseg && c0 >= sbase + a.seg[s].cnt) { sbase += a.seg[s].cnt; ++s; }
    const rsrc_t rs = s == 0 ? seg_rs[0] : (s == 1 ? seg_rs[1] : seg_rs[2]);
    const int stride = a.seg[s].stride;
    const int dy = kh - a.PH, dx = kw - a.PW;
    const int dpix = dy * a.W + dx;
    const int coff = c0 - sbase;
    const uint32_t base = lds0 + (uint32_t)(buf * STAGE * 16);
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int yy = a_y[j] + dy, xx = a_x[j] + dx;
      const bool ok = (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      const uint32_t off = (uint32_t)(((a_pix[j] + dpix) * stride + coff + a_lc[j]) * 2);
      raft_dma16(rs, base + j * NT * 16, ok ? off : OOB);
    }
    const uint32_t kb = (uint32_t)((tap * a.cin_pad + c0) * 2);
#pragma unroll
    for (int j = 0; j < B_PER; ++j)
      raft_dma16(w_rs, base + (A_CHUNKS + j * NT) * 16, b_off[j] == OOB ? OOB : b_off[j] + kb);
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto compute_upfront = [&](int buf) {
    const uint4* As = smem + buf * STAGE;
    const uint4* Bs = As + A_CHUNKS;
    bf16x8_t af[BK / 16][TM], bfr[BK / 16][TN];
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + (lane & 31);
        bfr[kk][j] = __builtin_bit_cast(bf16x8_t, Bs[swz(row, kk * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + (lane & 31);
        af[kk][i] = __builtin_bit_cast(bf16x8_t, As[swz(row, kk * 2 + (lane >> 5))]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, (BK / 16) * (TM + TN), 0);
    __builtin_amdgcn_sched_group_barrier(0x008, (BK / 16) * TM * TN, 0);
  };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < steps) issue(s, s);
  int cur = 0;
  for (int t = 0; t < steps; ++t) {
    const int newer = min(NS - 2, steps - 1 - t);
    if (NS >= 4 && newer >= 2) raft_wait_vmcnt<(NS >= 4 ? 2 : 0) * LPS>();
    else if (NS >= 3 && newer >= 1) raft_wait_vmcnt<(NS >= 3 ? 1 : 0) * LPS>();
    else raft_wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (t == 0) t1 = __builtin_amdgcn_s_memtime();
    if (t + NS - 1 < steps) {
      int nb = cur + NS - 1;
      nb = nb >= NS ? nb - NS : nb;
      issue(t + NS - 1, nb);
    }
    compute_upfront(cur);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }
  // force the MFMAs to complete before the stamp (read one accumulator)
  float sink = acc[0][0][0];
  asm volatile("" :: "v"(sink));
  t2 = __builtin_amdgcn_s_memtime();
  conv_epilogue<TM, TN, WM, WN, EPI>(a, acc, m0, n0, wm, wn, lane, P, HW);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  if (tid == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* o = st + (size_t)blockIdx.x * 6;
    o[0] = t0; o[1] = t1; o[2] = t2; o[3] = t3; o[4] = xcc;
    unsigned hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    o[5] = hwid;
  }
}

static float frand(unsigned& s) { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f; }
static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7FFF + ((u >> 16) & 1); return (uint16_t)(u >> 16); }

struct Geo { const char* name; int cout, KH, KW, nseg, segc[3]; };

int main(int argc, char** argv) {
  const int B = 12, H = 46, W = 62, P = B * H * W;
  Geo geos[] = {{"zr1", 256, 1, 5, 2, {128, 128, 0}}, {"q1", 128, 1, 5, 2, {128, 128, 0}},
                {"c2", 192, 3, 3, 1, {256, 0, 0}}};
  unsigned seed = 1;
  // inputs: one 256-channel bf16 buffer (segments are slices of it)
  std::vector<uint16_t> hin((size_t)P * 256);
  for (auto& v : hin) v = f2bf(frand(seed));
  uint16_t* din; CK(hipMalloc(&din, hin.size() * 2)); CK(hipMemcpy(din, hin.data(), hin.size() * 2, hipMemcpyHostToDevice));
  std::vector<uint16_t> hw((size_t)512 * 9 * 256);
  for (auto& v : hw) v = f2bf(0.05f * frand(seed));
  uint16_t* dw; CK(hipMalloc(&dw, hw.size() * 2)); CK(hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  float* dbias; CK(hipMalloc(&dbias, 1024 * 4)); CK(hipMemset(dbias, 0, 1024 * 4));
  void* dout; CK(hipMalloc(&dout, (size_t)P * 576 * 4));
  unsigned long long* dst; CK(hipMalloc(&dst, (size_t)4096 * 256 * 8));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (const Geo& g : geos) {
    ConvFwdArgs a{};
    int off = 0;
    for (int q = 0; q < g.nseg; ++q) { a.seg[q] = Seg{din + off, 256, g.segc[q]}; off += g.segc[q]; }
    a.nseg = g.nseg; a.cin_pad = off; a.cin_small = 0;
    a.B = B; a.H = H; a.W = W; a.KH = g.KH; a.KW = g.KW; a.PH = g.KH / 2; a.PW = g.KW / 2;
    a.wpk = dw; a.kpad = g.KH * g.KW * off; a.bias = dbias; a.cout = g.cout;
    a.out0 = dout; a.out0_stride = (g.cout + 63) / 64 * 64; a.scale = 1.f;
    const double flop = 2.0 * P * g.cout * a.kpad;
    printf("== %s cout %d K %d  (%.1f GF)\n", g.name, g.cout, a.kpad, flop * 1e-9);
    for (int idx : {16, 25, 26}) {
      float best = 1e30f;
      for (int trial = 0; trial < 3; ++trial) {
        if (!launch_conv_glds(a, EPI_BF16, idx, s)) break;
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < 10; ++r) launch_conv_glds(a, EPI_BF16, idx, s);
        CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms / 10);
      }
      if (best < 1e29f) printf("  cfg %2d: %7.1f us  %6.1f TF/s\n", idx, best * 1e3, flop / best * 1e-9);
    }
    // v3 kernels vs the LDS-DMA kernel of cfg 16 (5x1x1): same MFMA order -> identical bits
    {
      const size_t on = (size_t)P * a.out0_stride;
      launch_conv_glds(a, EPI_BF16, 16, s);
      CK(hipStreamSynchronize(s));
      std::vector<uint16_t> ref(on), got(on);
      CK(hipMemcpy(ref.data(), dout, on * 2, hipMemcpyDeviceToHost));
      auto v3 = [&](const char* tag, auto kern, int BM, int BN) {
        const int grid = conv_grid_1d(raft_cdiv(P, BM), raft_cdiv(a.cout, BN));
        CK(hipMemset(dout, 0xFF, on * 2));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), 0, s, a, (unsigned long long*)nullptr);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(got.data(), dout, on * 2, hipMemcpyDeviceToHost));
        size_t bad = 0;
        int shown = 0;
        std::vector<int> tiles;
        auto bf = [](uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; };
        for (int m = 0; m < P; ++m)
          for (int n = 0; n < g.cout; ++n)
            if (got[(size_t)m * a.out0_stride + n] != ref[(size_t)m * a.out0_stride + n]) {
              ++bad;
              if (shown < 6 && strcmp(tag, "5x1 o2") == 0) {
                printf("    mismatch m=%d (tile %d row %d) n=%d ref %g got %g\n", m, m / BM, m % BM, n,
                       bf(ref[(size_t)m * a.out0_stride + n]), bf(got[(size_t)m * a.out0_stride + n]));
                ++shown;
              }
              if (tiles.empty() || tiles.back() != m / BM) tiles.push_back(m / BM);
            }
        if (bad && strcmp(tag, "5x1 o2") == 0) {
          printf("    bad tiles %zu:", tiles.size());
          for (size_t i = 0; i < tiles.size() && i < 40; ++i) printf(" %d", tiles[i]);
          printf("\n");
        }
        float best = 1e30f;
        for (int trial = 0; trial < 3; ++trial) {
          CK(hipEventRecord(e0, s));
          for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), 0, s, a, (unsigned long long*)nullptr);
          CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms / 10);
        }
        printf("  v3 %-8s %7.1f us  %6.1f TF/s  mismatches %zu\n", tag, best * 1e3, flop / best * 1e-9, bad);
      };
      v3("5x1 o2", conv_fwd_v3_kernel<5, 1, EPI_BF16, 2>, 160, 128);
      v3("5x1 noA", conv_fwd_v3_kernel<5, 1, EPI_BF16, 2, false, 1>, 160, 128);
      v3("5x1 noB", conv_fwd_v3_kernel<5, 1, EPI_BF16, 2, false, 2>, 160, 128);
      v3("5x1 noAB", conv_fwd_v3_kernel<5, 1, EPI_BF16, 2, false, 3>, 160, 128);
      v3("4x1 o2", conv_fwd_v3_kernel<4, 1, EPI_BF16, 2>, 128, 128);
      v3("3x1 o2", conv_fwd_v3_kernel<3, 1, EPI_BF16, 2>, 96, 128);
      v3("2x1 o2", conv_fwd_v3_kernel<2, 1, EPI_BF16, 2>, 64, 128);
      v3("5x2 o1", conv_fwd_v3_kernel<5, 2, EPI_BF16, 1>, 160, 256);
      v3("3x2 o2", conv_fwd_v3_kernel<3, 2, EPI_BF16, 2>, 96, 256);
      v3("2x2 o2", conv_fwd_v3_kernel<2, 2, EPI_BF16, 2>, 64, 256);
      // per-step phase stamps of the 5x1 s4 kernel (wave 0 of every workgroup)
      {
        const int grid = conv_grid_1d(raft_cdiv(P, 160), raft_cdiv(a.cout, 128));
        CK(hipMemset(dst, 0, (size_t)4096 * 256 * 8));
        for (int r = 0; r < 3; ++r)
          hipLaunchKernelGGL((conv_fwd_v3_kernel<5, 1, EPI_BF16, 2, true>), dim3(grid), dim3(NT), 0, s, a, dst);
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h((size_t)grid * 256);
        CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
        const int steps = a.KH * a.KW * (a.cin_pad / 64);
        const int ns = std::min(60, steps);
        std::vector<double> pro, mainl, epi, sl0, dma, rest;
        for (int b = 0; b < grid; ++b) {
          const unsigned long long* o = &h[(size_t)b * 256];
          if (!o[0]) continue;
          pro.push_back(double(o[1] - o[0])); mainl.push_back(double(o[2] - o[1])); epi.push_back(double(o[3] - o[2]));
          for (int t = 1; t + 1 < ns; ++t) {
            sl0.push_back(double(o[5 + 4 * t] - o[4 + 4 * t]));
            dma.push_back(double(o[6 + 4 * t] - o[5 + 4 * t]));
            rest.push_back(double(o[4 + 4 * (t + 1)] - o[6 + 4 * t]));
          }
        }
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
        printf("  stamps 5x1: prologue %.0f main %.0f (%d steps) epi %.0f | per step: slice0 %.0f dma %.0f rest %.0f (MFMA floor %d/step)\n",
               med(pro), med(mainl), steps, med(epi), med(sl0), med(dma), med(rest), 20 * 32);
      }
    }
    if (getenv("LAB_STAMP") == nullptr) continue;
    // instrumented 5x1x1 (occ 1 and 2) and 5x2x1
    auto stamp = [&](const char* tag, auto kern, int BM, int BN) {
      const int grid = conv_grid_1d(raft_cdiv(P, BM), raft_cdiv(a.cout, BN));
      CK(hipMemset(dst, 0, 4096 * 6 * 8));
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), 0, s, a, dst);
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), 0, s, a, dst);
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10;
      std::vector<unsigned long long> h((size_t)grid * 6);
      CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long tmin = ~0ull, tmax = 0;
      std::vector<double> pro, mainl, epi, start;
      for (int b = 0; b < grid; ++b) { if (!h[b * 6]) continue; tmin = std::min(tmin, h[b * 6]); tmax = std::max(tmax, h[b * 6 + 3]); }
      for (int b = 0; b < grid; ++b) {
        const unsigned long long* o = &h[b * 6];
        if (!o[0]) continue;
        pro.push_back(double(o[1] - o[0])); mainl.push_back(double(o[2] - o[1])); epi.push_back(double(o[3] - o[2]));
        start.push_back(double(o[0] - tmin));
      }
      auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
      auto mx = [](std::vector<double> v) { return v.empty() ? 0.0 : *std::max_element(v.begin(), v.end()); };
      printf("  %-10s %7.1f us  WGs %zu  span %.0f cyc | prologue med %.0f max %.0f | main med %.0f max %.0f | epi med %.0f max %.0f | start max %.0f\n",
             tag, ms * 1e3, pro.size(), double(tmax - tmin), med(pro), mx(pro), med(mainl), mx(mainl), med(epi), mx(epi), mx(start));
    };
    stamp("5x1 occ1", conv_stamp_kernel<5, 1, 1, EPI_BF16, 2, 1>, 160, 128);
    stamp("5x1 occ2", conv_stamp_kernel<5, 1, 1, EPI_BF16, 2, 2>, 160, 128);
    stamp("5x2 occ1", conv_stamp_kernel<5, 2, 1, EPI_BF16, 2, 1>, 160, 256);
    stamp("2x2x2 o2", conv_stamp_kernel<2, 2, 2, EPI_BF16, 2, 2>, 128, 128);
    stamp("4x1 occ2", conv_stamp_kernel<4, 1, 1, EPI_BF16, 2, 2>, 128, 128);
  }
  return 0;
}
