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
void launch_corr_pyr_grad_reduce(float* const* glvl, const int* hs, const int* ws, int64_t planes,
                                 int levels, float inv_sqrt_c, float* out, hipStream_t stream);

// ---- window lookup (corr_lookup.hip); return false for an unsupported radius
bool launch_corr_lookup_fwd(const float* const* lvl, const int* hs, const int* ws, int levels,
                            const float* coords, float* out, int B, int H, int W, int radius,
                            hipStream_t stream);
bool launch_corr_lookup_bwd(float* const* glvl, const int* hs, const int* ws, int levels,
                            const float* coords, const float* dout, int B, int H, int W, int radius,
                            hipStream_t stream);

// ---- on-the-fly correlation (corr_onthefly.hip)
bool launch_corr_otf_fwd(const float* f1, const float* const* f2lvl, const int* hs, const int* ws,
                         int levels, const float* coords, float* out, int B, int C, int H, int W,
                         int radius, hipStream_t stream);
bool launch_corr_otf_bwd(const float* f1, const float* const* f2lvl, const int* hs, const int* ws,
                         int levels, const float* coords, const float* dout, float* df1,
                         float* const* df2lvl, int B, int C, int H, int W, int radius,
                         hipStream_t stream);

// ---- convex upsample (upsample.hip)
bool launch_convex_up_fwd(const float* flow, const void* mask, int mask_is_bf16, float* out, int B,
                          int H, int W, hipStream_t stream);
bool launch_convex_up_bwd(const float* flow, const void* mask, int mask_is_bf16, const float* dout,
                          void* dmask, float* wbuf, float* dflow, int B, int H, int W,
                          hipStream_t stream);

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
