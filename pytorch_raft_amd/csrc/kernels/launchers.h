// Host-side launch entry points of the gfx950 kernels (no torch types: raw pointers + stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#define RAFT_MAX_PREDS 32
struct PredPtrs {
  const float* p[RAFT_MAX_PREDS];
};
struct PredPtrsMut {
  float* p[RAFT_MAX_PREDS];
};

// ---- all-pairs correlation (corr_allpairs.hip)
void launch_corr_build(const float* f1, const float* f2, float* const* lvl, const int* hs,
                       const int* ws, int B, int C, int H, int W, int levels, hipStream_t stream);
// bf16 NHWC fmaps (B,H,W,C), C % 16 == 0
void launch_corr_build_bf16(const uint16_t* f1, const uint16_t* f2, void* const* lvl, const int* hs,
                            const int* ws, int B, int C, int H, int W, int levels, bool pyr_bf16,
                            hipStream_t stream);
void launch_corr_pyr_grad_reduce(float* const* glvl, const int* hs, const int* ws, int64_t planes,
                                 int levels, float inv_sqrt_c, float* out, hipStream_t stream);

// ---- window lookup (corr_lookup.hip); return false for an unsupported radius
bool launch_corr_lookup_fwd(const float* const* lvl, const int* hs, const int* ws, int levels,
                            const float* coords, void* out, int out_bf16, int64_t bs, int64_t ps,
                            int64_t cs, int B, int H, int W, int radius, hipStream_t stream);
bool launch_corr_lookup_bwd(float* const* glvl, const int* hs, const int* ws, int levels,
                            const float* coords, const float* dout, int64_t bs, int64_t ps,
                            int64_t cs, int B, int H, int W, int radius, hipStream_t stream);

// ---- on-the-fly correlation (corr_onthefly.hip); fmaps are NHWC bf16, out / dout (B,H,W,stride)
// f1lo / f2lo (nullable): bf16 low parts -> fp32-accurate split-bf16 forward
bool launch_corr_otf_fwd(const uint16_t* f1, const uint16_t* const* f2lvl, const uint16_t* f1lo,
                         const uint16_t* const* f2lo, const int* hs, const int* ws, int levels,
                         const float* coords, void* out, int out_bf16, int ostride, int B, int C,
                         int H, int W, int radius, hipStream_t stream);
bool launch_corr_otf_bwd(const uint16_t* f1, const uint16_t* const* f2lvl, const int* hs,
                         const int* ws, int levels, const float* coords, const void* dout,
                         int dout_bf16, int dstride, float* df1, float* const* df2lvl, int B,
                         int C, int H, int W, int radius, float* const* slab, const int* cap,
                         int* boxes, int dslo, hipStream_t stream);

// all iterations of a step at once from compact window gradients (see corr_window.hip)
struct WinList;
// slab / cap / boxes (nullable): deterministic dF2 -- per-tile slab rows [tile][cap[l]][C] fp32
// per level, boxes [tiles][4][4] int, then a fixed-order reduce (corr_otf_df2_reduce_kernel)
int otf_tiles(int B, int H, int W);
bool launch_corr_otf_window_bwd(const uint16_t* f1, const uint16_t* const* f2lvl, const int* hs,
                                const int* ws, int levels, const WinList& wl, float* df1,
                                float* const* df2lvl, int B, int C, int H, int W, int radius,
                                float* const* slab, const int* cap, int* boxes, float* df1b,
                                hipStream_t stream);

// ---- convex upsample (upsample.hip)
// mask element (b, ch, y, x) at b*mbs + ch*mcs + (y*W+x)*mps  (NCHW: mcs=HW, mps=1; NHWC: mcs=1, mps=576)
bool launch_convex_up_fwd(const float* flow, const void* mask, int mask_is_bf16, int64_t mbs,
                          int64_t mcs, int64_t mps, float* out, int B, int H, int W,
                          hipStream_t stream);
bool launch_convex_up_bwd(const float* flow, const void* mask, int mask_is_bf16, int64_t mbs,
                          int64_t mcs, int64_t mps, const float* dout, void* dmask, float* wbuf,
                          float* dflow, int B, int H, int W, hipStream_t stream);

// ---- sequence loss (loss.hip)
int seq_loss_partial_count();
void launch_seq_loss_fwd(const PredPtrs& preds, int n, const float* gt, const float* valid,
                         float gamma, float max_flow, int B, int64_t HW, float* partial, float* out,
                         hipStream_t stream);
void launch_seq_loss_bwd(const PredPtrs& preds, const PredPtrsMut& grads, int n, const float* gt,
                         const float* valid, const float* dloss, float gamma, float max_flow, int B,
                         int64_t HW, hipStream_t stream);

// ---- flow warping sampler (sampler.hip)
void launch_warp_fwd(const float* img, const float* flow, float* out, int B, int C, int H, int W,
                     float sx, float bx, float sy, float by, hipStream_t stream);
void launch_warp_bwd(const float* img, const float* flow, const float* dout, float* dimg,
                     float* dflow, int B, int C, int H, int W, float sx, float bx, float sy,
                     float by, hipStream_t stream);

// ---- implicit-GEMM convolution (conv_igemm.hip / conv_wgrad.hip)
enum ConvEpilogue {
  EPI_BF16 = 0,       // out0 bf16 = (acc + bias) * scale
  EPI_RELU_BF16 = 1,  // out0 bf16 = relu(acc + bias)
  EPI_F32 = 2,        // out0 f32 = (acc + bias) * scale
  EPI_ACC_F32 = 3,    // out0 f32 += (acc + bias) * scale
  EPI_GRU_ZR = 4,     // n < split: out0 = sigmoid (z); else out1 = sigmoid * aux0 (r*h), out2 = r
  EPI_GRU_Q = 5,      // q = tanh; out0 = aux0 + aux1 * (q - aux0) (h'), out1 = q
  EPI_DGRAD = 6,      // output channels split over oseg[] fp32 buffers (store or accumulate)
  EPI_F32_NCHW = 7,   // out0 f32 NCHW (B, cout, H, W)
  EPI_DGRAD_GATE = 8, // EPI_DGRAD + the fused ConvGRU gate backward (OSeg.gate); its own
                      // instantiation: the gate math's registers stay out of the plain dgrads
  // operand-type flag OR-ed into an epilogue id: every 16-bit operand / output of the conv is
  // fp16 (v_mfma_f32_32x32x16_f16; fp16 autocast) instead of bf16.  The names above say "BF16"
  // for "16-bit operand type".  LDS-DMA and halo kernels only (the register-staged configs
  // are bf16-only)
  EPI_F16 = 16,
  // split-fp32 flag (the fp32 schedule): every 16-bit activation the epilogue reads or writes is
  // an fp32 value carried as a bf16 pair -- hi at channel c, lo = bf16(v - hi) at channel
  // c + stride / 2 of the same pixel row -- and the conv runs with ConvFwdArgs.spl (K read as
  // [hi | lo | hi] against packed weights [w_hi | w_hi | w_lo]: three bf16 products, fp32
  // accumulation).  LDS-DMA and halo kernels only
  EPI_SPL = 32,
};
inline constexpr int epi_kind(int epi) { return epi & 15; }
inline constexpr bool epi_f16(int epi) { return (epi & EPI_F16) != 0; }
inline constexpr bool epi_spl(int epi) { return (epi & EPI_SPL) != 0; }
// operand type of the epilogue's 16-bit loads / stores: 0 bf16, 1 fp16, 2 split bf16 pair
inline constexpr int epi_ot(int epi) { return epi_f16(epi) ? 1 : (epi_spl(epi) ? 2 : 0); }

struct Seg {
  const uint16_t* ptr;  // bf16 NHWC base, already offset to the segment's first channel
  int stride;           // elements between consecutive pixels
  int cnt;              // channels (multiple of 32 unless SMALLC)
  int real;             // channels present (<= cnt, multiple of 8): the forward / dgrad kernels
                        // read the rest of the segment's K slot as zeros (a 96-channel tensor
                        // runs with a 128-channel K slot whose padded weights are zero)
};

struct OSeg {
  float* ptr;  // fp32 NHWC base offset to the segment's first channel (null: discard)
  int stride;
  int cnt;     // channel slots of this segment in the conv's output
  int real;    // channels actually written (< cnt for zero-padded slots)
  int acc;     // 1: +=, 0: =
  // relu-gated bf16 mode (ob != null): ob = bf16(ry > 0 ? v : 0) -- the gradient w.r.t. the
  // pre-activation of a ReLU whose output ry is this segment's forward input (fuses relu_bwd)
  uint16_t* ob;
  int ob_stride;
  const uint16_t* ry;
  int ry_stride;
  // fused ConvGRU gate backward on an fp32 segment (gate != 0; the segment itself is not
  // stored), per element (pixel, channel c < real) with v the dgrad value:
  //  gate 1 -- q / z gates on the state gradient g = *ptr + v (the final dh of a half-step):
  //            gb[c] = bf16(g z (1 - q^2)) (d pre-q), gz[c] = bf16(g (q - h) z (1 - z)) (d pre-z),
  //            gf1[c] = g (1 - z)                                   (ga0, ga1, ga2 = z, q, h)
  //  gate 2 -- r gate on d(r*h) = v: gb[real + c] = bf16(v h r (1 - r)), gf1[c] += v r
  //                                                               (ga1, ga2 = r, h)
  //  gate 3 -- the last accumulation into an fp32 gradient + the backward of the ReLU that
  //            produced this conv's input (ga0 = its output y): gb[c] = bf16([y > 0](gf1[c] + v))
  int gate;
  const uint16_t* ga0;
  const uint16_t* ga1;
  const uint16_t* ga2;
  int ga_stride;
  uint16_t* gb;
  int gb_stride;
  uint16_t* gz;
  int gz_stride;
  float* gf1;
  int gf_stride;
  // K prefix: this segment's columns read only the first kcin input channels (the rest of the
  // packed K is zero for them); 0 = all.  A workgroup whose N tile lies in such segments runs
  // only those K steps (one launch = two GEMMs sharing M and the leading K)
  int kcin;
};

struct ConvFwdArgs {
  Seg seg[3];
  int nseg;
  int cin_pad;    // sum of segment channel counts (multiple of 32)
  int cin_small;  // SMALLC: true input channels (K = KH*KW*cin_small densely packed)
  int B, H, W, KH, KW, PH, PW;
  const uint16_t* wpk;  // packed weights [Npad][kpad] bf16
  int kpad;
  const float* bias;    // may be null
  // GRU epilogues: per-pixel fp32 bias map [P][bmap_stride] added instead of `bias` (the
  // iteration-invariant context part of the ConvGRU convs, precomputed once per forward)
  const float* bmap;
  int bmap_stride;
  int bmap_bf16;        // 1: the bias map is bf16 (bmap points at uint16 data)
  int cout;
  void* out0;
  int out0_stride;
  void* out1;
  int out1_stride;
  void* out2;
  int out2_stride;
  const uint16_t* aux0;
  int aux0_stride;
  const uint16_t* aux1;
  int aux1_stride;
  float scale;
  int split;
  OSeg oseg[3];
  int noseg;
  int kprefix;  // 1: some output segment has kcin != 0 (per-tile K steps, tile_nchunk)
  // split-fp32 operands (set with EPI_SPL; the K map is compiled into the EPI_SPL
  // instantiations only): cin_pad = 3 x the segments' channel sum (a multiple of 64 each
  // third); K thirds 0 and 2 read the segments' hi halves, third 1 their lo halves (+ stride / 2)
  int spl;
};

// tile shape chosen per geometry: autotuned once (outside stream capture) and cached;
// RAFT_CONV_CFG=<idx> forces a config, RAFT_CONV_AUTOTUNE=0 uses the analytic heuristic
bool launch_conv_fwd(const ConvFwdArgs& a, int epi, int bn, bool smallc, hipStream_t stream);
// LDS-DMA kernel of config `idx` (conv_glds.hip); false for a non-LDS-DMA index
bool launch_conv_glds(const ConvFwdArgs& a, int epi, int idx, hipStream_t stream);
// rows of 13 ints: P H W KH KW cin cout small epi_class cfg BM BN channels-present
int conv_tuned_table(int* out, int max_rows);
// tests: run every following conv launch with config `idx` (-1: back to the tuned choice)
void conv_set_forced_cfg(int idx);
// data parallel: ranks > 0 skip the autotune (mode 0) and import rank 0's table (rows as
// conv_tuned_table), so every rank runs the same kernels; -1 restores RAFT_CONV_AUTOTUNE
void conv_set_autotune(int mode);
int conv_autotune_runs();
int conv_import_tuned(const int* rows, int n);

struct ConvWgradArgs {
  const uint16_t* g;  // dL/d(pre-activation), NHWC bf16, offset to channel 0
  int g_stride;
  Seg seg[3];
  int nseg;
  int cin_pad;
  int cin_small;
  int B, H, W, KH, KW, PH, PW;
  int cout;
  float* dw;  // [cout][kpad] fp32, accumulated
  int kpad;
  int pix_per_split;
  int splits_per_item;  // multi-item kernel: blockIdx.y = item * splits_per_item + split
  uint32_t w_magic;     // ceil(2^32 / W): q = umulhi(n, w_magic) = n / W for n * W < 2^32
  int f16;              // 1: fp16 operands (v_mfma_f32_32x32x16_f16), 0: bf16
};

// the iterations of one step whose weight gradients are summed by one launch
#define RAFT_WG_MAX_ITEMS 32
struct WgradItems {
  const uint16_t* g[RAFT_WG_MAX_ITEMS];       // dL/d(pre-activation), offset to channel 0
  const uint16_t* seg[RAFT_WG_MAX_ITEMS][3];  // forward input segments, offset to first channel
  int n;
};
bool launch_conv_wgrad_multi(const ConvWgradArgs& a, const WgradItems& it, int bm, float* db,
                             hipStream_t stream);

// tap-fused multi-item weight gradient (conv_wgrad_taps.hip): workgroup = (128 Cout) x (64 Cin) x
// all taps over a range of 8x8-pixel chunks; partial tiles go to a workspace and are reduced
#define RAFT_WG_MAX_CI_CHUNKS 16
struct WgradTapArgs {
  int n_ci;                              // 64-wide Cin chunks
  int ci_seg[RAFT_WG_MAX_CI_CHUNKS];     // input segment of each chunk
  int ci_off[RAFT_WG_MAX_CI_CHUNKS];     // channel offset inside the segment
  int ci_k[RAFT_WG_MAX_CI_CHUNKS];       // packed-K column of the chunk's first channel (tap 0)
  int ci_cnt[RAFT_WG_MAX_CI_CHUNKS];     // valid channels of the chunk (64, or a 32 tail)
  int bm;                                // Cout tile: 128, or 64 (3x3 with Cout <= 64)
  int n_co;                              // Cout tiles
  int tiles_x, tiles_per_img, chunks_per_item, total_chunks, chunks_per_split, splits;
  float* w_part;                         // [splits][cout][kpad]
  float* db_part;                        // [splits][cout] or null
  uint16_t* dw_bf16;                     // non-null: dW stored as bf16 here (no accumulate)
  int dw_f16;                            // ... as fp16 instead (fp16 autocast)
  int db_items;                          // > 0: only items < db_items add to the bias gradient
};
bool launch_conv_wgrad_taps(const ConvWgradArgs& a, const WgradItems& it, const WgradTapArgs& ta,
                            float* db, hipStream_t stream);

// db (nullable): fp32 bias gradient += column sums of G (fused)
bool launch_conv_wgrad(const ConvWgradArgs& a, int bm, bool smallc, float* db, hipStream_t stream);
void launch_col_sum(const uint16_t* g, int stride, int cout, int P, float* db, hipStream_t stream);

// ---- fused update-block elementwise kernels (update_ew.hip)
// empty kernel `raft_phase_marker_kernel` (trace phase boundaries, scripts/prof_diff.py --phases)
void launch_phase_marker(hipStream_t stream);
// stride-1 3x3 64 -> 64 NHWC bf16 conv (conv_enc64.hip); wpk = (64, 9*64) packed [n][tap*64 + c]
// encoder stem conv (stem_conv.hip): 7x7 stride 2 pad 3, 3 -> C (64 / 32) channels, NHWC 16-bit;
// w = the (C, 7, 7, 3)-ordered weight; out (B, Ho, Wo, C); grid = persistent workgroups
int stem_conv_tiles(int B, int Ho, int Wo);
bool launch_stem_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* out, int B, int H, int W,
                          int Ho, int Wo, int C, int grid, int f16, hipStream_t stream);
// weight gradient: part = grid x C x 224 fp32 scratch, dw = (C, 7, 7, 3) 16-bit result
bool launch_stem_conv_wgrad(const uint16_t* x, const uint16_t* gy, float* part, uint16_t* dw, int B,
                            int H, int W, int Ho, int Wo, int C, int grid, int f16, hipStream_t stream);
// part != null: per-tile norm statistics [tile][4][64] (sum(x-K), sum((x-K)^2), K, count), tiles
// image-major, ceil(H/8) x ceil(W/16) per image (conv_enc64_tiles)
bool launch_conv_enc64(const uint16_t* x, const uint16_t* wpk, uint16_t* out, int B, int H, int W,
                       int grid_cap, int f16, hipStream_t stream, float* part = nullptr);
inline int conv_enc64_tiles(int H, int W) { return ((H + 7) / 8) * ((W + 15) / 16); }
// fp32 (B,C,H,W) any strides -> (B,H,W,2cp) bf16 [hi | lo], zero padded (ops/conv_fp32.py)
void launch_split_hilo(const float* x, int64_t sb, int64_t sc, int64_t sh, int64_t sw, int B, int C,
                       int H, int W, int cp, uint16_t* out, hipStream_t stream);
void launch_relu_bwd(const float* g, int gs, const uint16_t* y, int ys, uint16_t* out, int os, int P,
                     int C, float scale, hipStream_t stream, int ot = 0);
// ot: 0 bf16, 1 fp16, 2 split fp32 (bf16 [hi | lo] row halves)
void launch_gru_q_bwd(const float* dh, const uint16_t* z, const uint16_t* q, const uint16_t* hprev,
                      uint16_t* dpre_q, float* dz, float* dhprev, int P, int hd, hipStream_t stream, int ot = 0);
void launch_gru_zr_bwd(const float* drh, const float* dz, const uint16_t* z, const uint16_t* r,
                       const uint16_t* hprev, uint16_t* dpre_zr, float* dhprev, int P, int hd,
                       hipStream_t stream, int ot = 0);
void launch_flow_prep(const float* flow, uint16_t* flowb, uint16_t* slot, int slot_stride, int B,
                      int HW, hipStream_t stream);
// out (bf16 or fp32) = sum of n <= RAFT_SUM_MAX bf16 tensors (+ fp32 carry); numel % 8 == 0
#define RAFT_SUM_MAX 32
struct BfPtrs {
  const uint16_t* p[RAFT_SUM_MAX];
};
void launch_sum_bf16(const BfPtrs& ins, int n, const float* carry, void* out, bool out_f32,
                     int64_t numel, int f16, hipStream_t stream);
// (B,2,H,W) fp32 flow -> (B,H,W,128) bf16 7x7 patch (tap-major, 2 ch), + optional flow slot
void launch_f1_patch(const float* flow, uint16_t* patch, uint16_t* slot, int slot_stride, int B, int H,
                     int W, int f16, hipStream_t stream);

// ---- flow_head.conv2 (3x3, 256 -> 2): fwd / dgrad (+ReLU gate) / multi-item wgrad (flow_head2.hip)
#define RAFT_FH2_MAX_ITEMS 32
struct Fh2Items {
  const float* gout[RAFT_FH2_MAX_ITEMS];    // (B,2,H,W) fp32 output gradient per iteration
  const uint16_t* in[RAFT_FH2_MAX_ITEMS];   // (B,H,W,cs) bf16 input (channels 0..255 used)
  int n;
};
// wf: bf16 pairs [t][o][c/2] (9*2*128 uint32); wd: bf16 pairs (W0[c], W1[c]) [t][c] (9*256 uint32)
// f16: fp16 activations / weight pairs (v_dot2_f32_f16) instead of bf16
// coords (optional, (B,2,H,W) fp32): also writes cnew = coords + out and fnew = cnew - (x, y)
bool launch_fh2_fwd(const uint16_t* in, int cs, const uint32_t* wf, const float* bias, float* out,
                    int B, int H, int W, int f16, hipStream_t stream, const float* coords = nullptr,
                    float* cnew = nullptr, float* fnew = nullptr);
bool launch_fh2_dgrad(const float* gout, const uint32_t* wd, const uint16_t* fm, int fs, uint16_t* dx,
                      int ds, int B, int H, int W, int f16, hipStream_t stream);
// part: (blocks, 2*2304 + 2) fp32 per-workgroup partial [dw | db] rows (fully written)
int fh2_wgrad_units(int n, int B, int H);
bool launch_fh2_wgrad(const Fh2Items& it, int cs, int B, int H, int W, float* part, int blocks,
                      int f16, hipStream_t stream);

// ---- NHWC lookup tile + window-compact backward (corr_window.hip)
#define RAFT_MAX_WIN 32
struct WinList {
  const float* coords[RAFT_MAX_WIN];   // (B,2,H,W) per iteration
  const float* wg[RAFT_MAX_WIN];       // (B,N,L,E,E) per iteration (corr_window_reduce)
  const uint16_t* dout[RAFT_MAX_WIN];  // (B,H,W,cbuf) bf16 tap gradients (on-the-fly backward)
  int cbuf;
  int n;
};
// out_f16: fp16 taps (fp32 pyramid only) instead of bf16
bool launch_corr_lookup_tile(const void* const* lvl, const int* hs, const int* ws, int levels,
                             const float* coords, uint16_t* out, int cbuf, int B, int H, int W,
                             int radius, bool pyr_bf16, int out_f16, hipStream_t stream);
bool launch_corr_window_grad(const float* coords, const uint16_t* dout, int cbuf, float* wg, int B,
                             int H, int W, int levels, int radius, hipStream_t stream);
struct TapList {
  const float* coords[RAFT_MAX_WIN];   // (B,2,H,W) per iteration
  const uint16_t* dout[RAFT_MAX_WIN];  // (B,H,W,cbuf) bf16 lookup-output gradient per iteration
  int cbuf;
  int n;
  int ldo;  // row pitch of the (B, N, ldo) output (elements, >= N, even for bf16 when N is);
            // columns N..ldo-1 are written as zeros (the MFMA backward GEMMs' K padding)
  int tf16; // 1: the tap gradients are fp16 (fp16 autocast), 0: bf16
};
int corr_tap_reduce_lds_bytes(int H, int W, int levels, int radius);
// list: (1 + B*H*W) ints of scratch for the box fold's overflow list (nullptr: no box fold)
bool launch_corr_tap_reduce(const TapList& tl, int levels, int B, int H, int W, int radius,
                            float inv_sqrt_c, void* out, int out_bf16, int* list, hipStream_t stream);
// all-pairs feature-map gradients (corr_bwd.hip): dc (B, N, ldc) bf16 from the fold (ldc % 64 ==
// 0, zero columns past N), f1 / f2 (B, N, C) bf16 NHWC, f2t scratch (B, C, ldc);
// g1 = dC F2, g2 = dC^T F1 as (B, N, C) bf16.  False for an unsupported geometry (C % 128 != 0)
bool launch_corr_bwd_fmaps(const uint16_t* dc, int ldc, const uint16_t* f1, const uint16_t* f2,
                           uint16_t* f2t, uint16_t* g1, uint16_t* g2, int B, int N, int C,
                           hipStream_t stream);
// fp32 correlation (split-bf16, three passes per GEMM): dc2 (2, B, N, ldc) bf16 [hi | lo] planes,
// f1 / f2 fp32 (B, C, N); scratch f2s (2, B, C, ldc), f1s (2, B, N, C) bf16; g1 / g2 fp32 (B, N, C)
bool launch_corr_bwd_fmaps_split(const uint16_t* dc2, int ldc, const float* f1, const float* f2,
                                 uint16_t* f2s, uint16_t* f1s, float* g1, float* g2, int B, int N, int C,
                                 hipStream_t stream);
int corr_window_reduce_lds_bytes(int H, int W, int levels);
// out: (B, N, N) fp32, or bf16 when out_bf16 (mixed-precision backward GEMMs)
bool launch_corr_window_reduce(const WinList& wl, int levels, int B, int H, int W, int radius,
                               float inv_sqrt_c, void* out, int out_bf16, hipStream_t stream);

// ---- NHWC convex upsample (upsample.hip)
bool launch_convex_up_nhwc_fwd(const float* flow, const void* mask, int mask_is_bf16, float* out,
                               int B, int H, int W, hipStream_t stream);
bool launch_convex_up_nhwc_bwd(const float* flow, const void* mask, int mask_is_bf16,
                               const float* dout, void* dmask, float* wbuf, float* dflow, int B,
                               int H, int W, hipStream_t stream);

// ---- encoder norm + activation, NHWC bf16 / fp16 (f16) (encoder_norm.hip)
// mode: 0 instance, 1 batch (training statistics), 2 batch (running statistics), 3 none
int encoder_norm_blocks(int64_t range, int C, int groups, int* pix_per_blk);
void launch_norm_stats(const uint16_t* x, int N, int HW, int C, int per_image, float* part,
                       int nblk, int pix_per_blk, int f16, hipStream_t stream);
// training statistics (mode 0 / 1) from a producing conv's per-tile rows [tile][4][C]
// (conv_enc64.hip); nblk = tiles per group (image for mode 0, the whole batch for mode 1)
void launch_norm_finalize_tiled(const float* part, int nblk, int N, int HW, int C, int mode,
                                const float* gamma, const float* beta, const float* cbias,
                                float* rmean, float* rvar, float momentum, float eps, float* mean,
                                float* invstd, float* scale, float* shift, hipStream_t stream);
void launch_norm_finalize(const float* part, const uint16_t* x, int N, int HW, int C, int mode,
                          int nblk, const float* gamma, const float* beta, const float* cbias,
                          float* rmean, float* rvar, float momentum, float eps, float* mean,
                          float* invstd, float* scale, float* shift, int f16, hipStream_t stream);
// ys (nullable, fp32 only): y also as the split-bf16 conv operand, (N*HW, 2 spad) [hi | lo]
void launch_norm_apply(const uint16_t* x, const float* scale, const float* shift, int N, int HW,
                       int C, int relu, const uint16_t* res, uint16_t* y, int f16, hipStream_t stream,
                       uint16_t* ys = nullptr, int spad = 0);
void launch_add_relu(const uint16_t* a, const uint16_t* b, uint16_t* out, int64_t n,
                     int f16, hipStream_t stream);
// context-encoder output: in (P pixels x C, NHWC) -> h = tanh(in[:, :hdim]) (P x hdim), x =
// relu(in[:, hdim:]) (P x (C - hdim)); bf16 / fp16 (f16); and its backward (gh / gx nullable)
void launch_ctx_act(const uint16_t* in, int64_t P, int C, int hdim, uint16_t* h, uint16_t* x, int f16,
                    hipStream_t stream);
void launch_ctx_act_bwd(const uint16_t* gh, const uint16_t* gx, const uint16_t* h, const uint16_t* x,
                        int64_t P, int C, int hdim, uint16_t* gin, int f16, hipStream_t stream);
// g = (dy [+ dy2]) * [y > 0]; dy2 nullable
void launch_relu_mask(const uint16_t* dy, const uint16_t* dy2, const uint16_t* y, uint16_t* g, int64_t n,
                      int f16, hipStream_t stream);
// y (nullable): the forward output; when given, the ReLU mask is read from it, else recomputed
// yres (nullable): dy is the gradient of a residual block's output relu(branch + res) = yres;
// g = (dy [+ dy2]) * [yres > 0] is formed in the statistics pass and stored to gout (the
// residual's gradient), and the norm backward runs on it (the block-end ReLU mask fused)
// dxs (nullable, fp32 only): dx also as the split-bf16 operand (N*HW, 2 spad) [hi | lo]
void launch_norm_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean,
                     const float* invstd,
                     int N, int HW, int C, int mode, int relu, const float* gamma,
                     const float* beta, float* part, int nblk, int pix_per_blk, float* coef,
                     float* dgamma, float* dbeta, float* dcbias, uint16_t* dx,
                     const uint16_t* dy2, const uint16_t* yres, uint16_t* gout, int f16, hipStream_t stream,
                     uint16_t* dxs = nullptr, int spad = 0);

// ---- multi-tensor AdamW + global-norm clip + GradScaler unscale / overflow skip (adamw.hip)
struct AdamTensor {
  float* p;
  float* g;
  float* m;
  float* v;
  int64_t numel;
  float* step;  // device step counter of this tensor (advanced on every finite step)
  int group;    // index into the AdamGroup table
};
struct AdamGroup {
  const float* lr_dev;  // nullable: lr from the device (graph-ready schedule)
  float lr, wd, b1, b2, omb1, omb2, eps;  // omb = 1 - beta computed in double on the host
};
int adam_chunk_elems();
// tab / cum / groups: device tables (T tensors, cum[T] = nchunks); part: nchunks floats;
// coef: 3 floats (gradient multiplier, total norm, found_inf); max_norm <= 0: no clipping;
// inv_scale (nullable): 1 / GradScaler scale; need_norm: run the sum-of-squares pass (clipping or
// overflow detection); found_inf (nullable): the GradScaler's flag, written
void launch_adamw_multi(const AdamTensor* tab, const int* cum, int T, int nchunks, const AdamGroup* groups,
                        float max_norm, const float* inv_scale, int need_norm, int write_grad,
                        float* part, float* coef, float* found_inf, hipStream_t stream);

// ---- gather.hip: multi-source gather + cast (per-step weight packing)
#define RAFT_GATHER_MAX 62   // sources per launch (index field 63 = the zero padding slot)
#define RAFT_GATHER_ZERO 63
struct GatherSrcs {
  const void* p[RAFT_GATHER_MAX];
  int n;
  int lo_from;   // sources k >= lo_from yield the split-fp32 residual v - bf16(v) (bf16 output)
};
// out[i] = cast(p[idx[i] >> 26][idx[i] & (2^26 - 1)]), 0 for the zero slot; it / ot (source /
// output type): 0 bf16, 1 fp16, 2 fp32 -- fp32 -> any, or bf16 / fp16 -> fp32
bool launch_gather_cast(const GatherSrcs& s, const int32_t* idx, void* out, int64_t n, int it, int ot,
                        hipStream_t stream);

// ---- image_prep.hip: both frames -> 2 * (x / 255) - 1 as one channels_last (2B,H,W,3) batch;
// ot: 0 bf16, 1 fp16, 2 fp32
bool launch_image_prep(const float* a, const float* b, void* out, int B, int64_t HW, int ot,
                       hipStream_t stream);
