// PPEG: pyramid positional encoding generator (code/models/TransMIL.py:60-75).
//
//   out = dw7x7(g) + g + dw5x5(g) + dw3x3(g)   on the G x G patch grid, zero padding,
//   per-channel biases; the class token (row 0) passes through.
//
// The three depthwise convolutions, the identity and the three biases fold into
// ONE 7x7 depthwise stencil (w = w7 + pad(w5) + pad(w3) + delta, b = b7+b5+b3),
// applied channel-last directly on the [B, S, D] fp32 residual stream: token
// t = 1 + r*G + c (row-major, :71).  No transpose to NCHW, no padded copy.
// Threads own (column group, channel): a wave covers 64 consecutive channels so
// every tap load is one 256-B coalesced row segment.  HBM-bound.
#include "common.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int KS = 7, R = 3, NT = 49;

// w_fold[ch][49], b_fold[ch]
__global__ void ppeg_fold_kernel(const float* __restrict__ w7, const float* __restrict__ b7,
                                 const float* __restrict__ w5, const float* __restrict__ b5,
                                 const float* __restrict__ w3, const float* __restrict__ b3, int D,
                                 float* __restrict__ wf, float* __restrict__ bf) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= D) return;
  for (int dy = 0; dy < KS; ++dy)
    for (int dx = 0; dx < KS; ++dx) {
      float v = w7[(size_t)ch * NT + dy * KS + dx];
      if (dy >= 1 && dy <= 5 && dx >= 1 && dx <= 5) v += w5[(size_t)ch * 25 + (dy - 1) * 5 + (dx - 1)];
      if (dy >= 2 && dy <= 4 && dx >= 2 && dx <= 4) v += w3[(size_t)ch * 9 + (dy - 2) * 3 + (dx - 2)];
      if (dy == R && dx == R) v += 1.0f;
      wf[(size_t)ch * NT + dy * KS + dx] = v;
    }
  bf[ch] = b7[ch] + b5[ch] + b3[ch];
}

// grid (G, B, D/64), block 256: thread (cg = tid>>6, ch = chunk*64 + lane)
template <bool BWD_DATA>
__global__ __launch_bounds__(256) void ppeg_stencil_kernel(const float* __restrict__ x, int S, int G, int D,
                                                           const float* __restrict__ wf, const float* __restrict__ bf,
                                                           float* __restrict__ y) {
  const int r = blockIdx.x, b = blockIdx.y, ch = blockIdx.z * 64 + (threadIdx.x & 63), cg = threadIdx.x >> 6;
  float w[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) w[t] = wf[(size_t)ch * NT + (BWD_DATA ? NT - 1 - t : t)];
  const float bias = BWD_DATA ? 0.f : bf[ch];
  const float* xb = x + (size_t)b * S * D + D + ch;  // grid token (0,0)
  float* yb = y + (size_t)b * S * D;
  if (r == 0 && cg == 0) yb[ch] = x[(size_t)b * S * D + ch];  // class token passes through
  for (int c = cg; c < G; c += 4) {
    float acc = bias;
#pragma unroll
    for (int dy = 0; dy < KS; ++dy) {
      const int rr = r + dy - R;
      if (rr < 0 || rr >= G) continue;
#pragma unroll
      for (int dx = 0; dx < KS; ++dx) {
        const int cc = c + dx - R;
        if (cc < 0 || cc >= G) continue;
        acc = fmaf(w[dy * KS + dx], xb[((size_t)rr * G + cc) * D], acc);
      }
    }
    yb[(size_t)(1 + r * G + c) * D + ch] = acc;
  }
}

// weight/bias gradient partials: part[(b*G + r)][ch*50 + t] (t = 49 -> bias)
__global__ __launch_bounds__(256) void ppeg_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy_,
                                                         int S, int G, int D, float* __restrict__ part) {
  const int r = blockIdx.x, b = blockIdx.y, ch = blockIdx.z * 64 + (threadIdx.x & 63), cg = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const float* xb = x + (size_t)b * S * D + D + ch;
  const float* gb = dy_ + (size_t)b * S * D + D + ch;
  float acc[NT + 1];
#pragma unroll
  for (int t = 0; t <= NT; ++t) acc[t] = 0.f;
  for (int c = cg; c < G; c += 4) {
    const float g = gb[((size_t)r * G + c) * D];
    acc[NT] += g;
#pragma unroll
    for (int dy = 0; dy < KS; ++dy) {
      const int rr = r + dy - R;
      if (rr < 0 || rr >= G) continue;
#pragma unroll
      for (int dx = 0; dx < KS; ++dx) {
        const int cc = c + dx - R;
        if (cc < 0 || cc >= G) continue;
        acc[dy * KS + dx] = fmaf(g, xb[((size_t)rr * G + cc) * D], acc[dy * KS + dx]);
      }
    }
  }
  __shared__ float red[4][64][NT + 1];
#pragma unroll
  for (int t = 0; t <= NT; ++t) red[cg][lane][t] = acc[t];
  __syncthreads();
  float* dst = part + ((size_t)b * G + r) * D * (NT + 1) + (size_t)blockIdx.z * 64 * (NT + 1);
  for (int e = threadIdx.x; e < 64 * (NT + 1); e += 256) {
    const int l = e / (NT + 1), t = e % (NT + 1);
    dst[e] = (red[0][l][t] + red[1][l][t]) + (red[2][l][t] + red[3][l][t]);
  }
}

// unfold folded gradients: dw7 = dwf, dw5 = centre 5x5, dw3 = centre 3x3, db* = db
__global__ void ppeg_unfold_kernel(const float* __restrict__ g, int D, float* __restrict__ dw7,
                                   float* __restrict__ db7, float* __restrict__ dw5, float* __restrict__ db5,
                                   float* __restrict__ dw3, float* __restrict__ db3) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= D) return;
  const float* s = g + (size_t)ch * (NT + 1);
  for (int t = 0; t < NT; ++t) dw7[(size_t)ch * NT + t] = s[t];
  for (int dy = 0; dy < 5; ++dy)
    for (int dx = 0; dx < 5; ++dx) dw5[(size_t)ch * 25 + dy * 5 + dx] = s[(dy + 1) * KS + dx + 1];
  for (int dy = 0; dy < 3; ++dy)
    for (int dx = 0; dx < 3; ++dx) dw3[(size_t)ch * 9 + dy * 3 + dx] = s[(dy + 2) * KS + dx + 2];
  db7[ch] = s[NT]; db5[ch] = s[NT]; db3[ch] = s[NT];
}

}  // namespace

extern "C" int tm_ppeg_fold(const float* w7, const float* b7, const float* w5, const float* b5, const float* w3,
                            const float* b3, int D, float* wfold, float* bfold, void* stream) {
  ppeg_fold_kernel<<<(D + 63) / 64, 64, 0, (hipStream_t)stream>>>(w7, b7, w5, b5, w3, b3, D, wfold, bfold);
  TM_CHECK_LAUNCH();
  return 0;
}

// x, y: [B, S, D] fp32 with S = 1 + G*G.  y must not alias x.
extern "C" int tm_ppeg_fwd(const float* x, int B, int G, int D, const float* wfold, const float* bfold, float* y,
                           void* stream) {
  TM_REQUIRE(x && y && x != y && D % 64 == 0 && G > 0, "ppeg_fwd: bad args");
  ppeg_stencil_kernel<false><<<dim3(G, B, D / 64), 256, 0, (hipStream_t)stream>>>(x, 1 + G * G, G, D, wfold, bfold, y);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_ppeg_bwd_workspace(int B, int G, int D) {
  return (long long)B * G * D * 50 * (long long)sizeof(float);
}

// dy: [B,S,D] upstream gradient; x: PPEG input.  dx written (=); weight grads written.
extern "C" int tm_ppeg_bwd(const float* x, const float* dy, int B, int G, int D, const float* wfold, float* dx,
                           float* work, float* dwsum, float* dw7, float* db7, float* dw5, float* db5, float* dw3,
                           float* db3, void* stream) {
  TM_REQUIRE(x && dy && dx && dx != dy && D % 64 == 0, "ppeg_bwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  const int S = 1 + G * G;
  ppeg_stencil_kernel<true><<<dim3(G, B, D / 64), 256, 0, st>>>(dy, S, G, D, wfold, nullptr, dx);
  TM_CHECK_LAUNCH();
  ppeg_wgrad_kernel<<<dim3(G, B, D / 64), 256, 0, st>>>(x, dy, S, G, D, work);
  TM_CHECK_LAUNCH();
  if (int rc = tm_splitk_reduce(work, dwsum, B * G, (long long)D * 50, 1.0f, 0, stream)) return rc;
  ppeg_unfold_kernel<<<(D + 63) / 64, 64, 0, st>>>(dwsum, D, dw7, db7, dw5, db5, dw3, db3);
  TM_CHECK_LAUNCH();
  return 0;
}
