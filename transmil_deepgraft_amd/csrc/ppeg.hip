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

// w_fold[49][ch] (tap-major: a wave's 64 channels of one tap are one 256-B load), b_fold[ch]
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
      wf[(size_t)(dy * KS + dx) * D + ch] = v;
    }
  bf[ch] = b7[ch] + b5[ch] + b3[ch];
}

// Register-blocked stencil: a thread owns one channel and a 4x4 block of grid
// cells; it streams the 10x10 input window once (100 loads, each a 256-B
// coalesced row segment across the wave's 64 channels) for 784 FMAs.
// grid (ceil(nCB/4) * D/64, nRB, B), block 256: wave w -> column block 4*bx + w.
constexpr int RB = 4;
constexpr int WRB = 4;  // row blocks per weight-gradient workgroup

template <bool BWD_DATA>
__global__ __launch_bounds__(256) void ppeg_stencil_kernel(const float* __restrict__ x, int S, int G, int D,
                                                           const float* __restrict__ wf, const float* __restrict__ bf,
                                                           float* __restrict__ y) {
  const int nchunk = D / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ch = (blockIdx.x % nchunk) * 64 + lane;
  const int cb = (blockIdx.x / nchunk) * 4 + wave;
  const int r0 = blockIdx.y * RB, c0 = cb * RB, b = blockIdx.z;
  float* yb = y + (size_t)b * S * D;
  if (blockIdx.x < (unsigned)nchunk && blockIdx.y == 0 && wave == 0) yb[ch] = x[(size_t)b * S * D + ch];  // class token
  if (c0 >= G) return;
  float w[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) w[t] = wf[(size_t)(BWD_DATA ? NT - 1 - t : t) * D + ch];
  const float bias = BWD_DATA ? 0.f : bf[ch];
  float acc[RB][RB];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < RB; ++j) acc[i][j] = bias;
  const float* xb = x + (size_t)b * S * D + D + ch;  // grid token (0,0)
#pragma unroll
  for (int ir = 0; ir < RB + KS - 1; ++ir) {
    const int rr = r0 - R + ir;
    if (rr < 0 || rr >= G) continue;
    float xv[RB + KS - 1];
#pragma unroll
    for (int ic = 0; ic < RB + KS - 1; ++ic) {
      const int cc = c0 - R + ic;
      xv[ic] = (cc >= 0 && cc < G) ? xb[((size_t)rr * G + cc) * D] : 0.f;
    }
#pragma unroll
    for (int orow = 0; orow < RB; ++orow) {
      const int dy = ir - orow;
      if (dy < 0 || dy >= KS) continue;
#pragma unroll
      for (int oc = 0; oc < RB; ++oc)
#pragma unroll
        for (int dx = 0; dx < KS; ++dx) acc[orow][oc] = fmaf(w[dy * KS + dx], xv[oc + dx], acc[orow][oc]);
    }
  }
#pragma unroll
  for (int orow = 0; orow < RB; ++orow)
#pragma unroll
    for (int oc = 0; oc < RB; ++oc) {
      const int r = r0 + orow, c = c0 + oc;
      if (r < G && c < G) yb[(size_t)(1 + r * G + c) * D + ch] = acc[orow][oc];
    }
}

// weight/bias gradient partials.  grid (ceil(nCB/4) * D/64, ceil(nRB/WRB), B), block 256:
// a thread owns a channel and walks WRB row blocks of its column block; partial slab
// index = (b * gridDim.y + by) * gridDim.x/nchunk + bx/nchunk, layout [slab][ch][50].
__global__ __launch_bounds__(256) void ppeg_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy_,
                                                         int S, int G, int D, float* __restrict__ part) {
  const int nchunk = D / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunk = blockIdx.x % nchunk, ch = chunk * 64 + lane;
  const int cb = (blockIdx.x / nchunk) * 4 + wave;
  const int c0 = cb * RB, b = blockIdx.z;
  const float* xb = x + (size_t)b * S * D + D + ch;
  const float* gb = dy_ + (size_t)b * S * D + D + ch;
  float acc[NT + 1];
#pragma unroll
  for (int t = 0; t <= NT; ++t) acc[t] = 0.f;
  if (c0 < G) {
    for (int rb = blockIdx.y * WRB; rb < blockIdx.y * WRB + WRB; ++rb) {
      const int r0 = rb * RB;
      if (r0 >= G) break;
      float gv[RB][RB];
#pragma unroll
      for (int orow = 0; orow < RB; ++orow)
#pragma unroll
        for (int oc = 0; oc < RB; ++oc) {
          const int r = r0 + orow, c = c0 + oc;
          gv[orow][oc] = (r < G && c < G) ? gb[((size_t)r * G + c) * D] : 0.f;
          acc[NT] += gv[orow][oc];
        }
#pragma unroll
      for (int ir = 0; ir < RB + KS - 1; ++ir) {
        const int rr = r0 - R + ir;
        if (rr < 0 || rr >= G) continue;
        float xv[RB + KS - 1];
#pragma unroll
        for (int ic = 0; ic < RB + KS - 1; ++ic) {
          const int cc = c0 - R + ic;
          xv[ic] = (cc >= 0 && cc < G) ? xb[((size_t)rr * G + cc) * D] : 0.f;
        }
#pragma unroll
        for (int orow = 0; orow < RB; ++orow) {
          const int dy = ir - orow;
          if (dy < 0 || dy >= KS) continue;
#pragma unroll
          for (int oc = 0; oc < RB; ++oc)
#pragma unroll
            for (int dx = 0; dx < KS; ++dx) acc[dy * KS + dx] = fmaf(gv[orow][oc], xv[oc + dx], acc[dy * KS + dx]);
        }
      }
    }
  }
  __shared__ float red[4][64][NT + 1];
#pragma unroll
  for (int t = 0; t <= NT; ++t) red[wave][lane][t] = acc[t];
  __syncthreads();
  const int slab = (b * gridDim.y + blockIdx.y) * (gridDim.x / nchunk) + blockIdx.x / nchunk;
  float* dst = part + (size_t)slab * D * (NT + 1) + (size_t)chunk * 64 * (NT + 1);
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
  const int ncb = (G + RB - 1) / RB;
  const dim3 grid(((ncb + 3) / 4) * (D / 64), ncb, B);
  ppeg_stencil_kernel<false><<<grid, 256, 0, (hipStream_t)stream>>>(x, 1 + G * G, G, D, wfold, bfold, y);
  TM_CHECK_LAUNCH();
  return 0;
}

static int ppeg_wgrad_slabs(int B, int G) {
  const int ncb = (G + RB - 1) / RB;
  return B * ((ncb + 3) / 4) * ((ncb + WRB - 1) / WRB);
}

extern "C" long long tm_ppeg_bwd_workspace(int B, int G, int D) {
  return (long long)ppeg_wgrad_slabs(B, G) * D * 50 * (long long)sizeof(float);
}

// dy: [B,S,D] upstream gradient; x: PPEG input.  dx written (=); weight grads written.
extern "C" int tm_ppeg_bwd(const float* x, const float* dy, int B, int G, int D, const float* wfold, float* dx,
                           float* work, float* dwsum, float* dw7, float* db7, float* dw5, float* db5, float* dw3,
                           float* db3, void* stream) {
  TM_REQUIRE(x && dy && dx && dx != dy && D % 64 == 0, "ppeg_bwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  const int S = 1 + G * G;
  const int ncb = (G + RB - 1) / RB;
  ppeg_stencil_kernel<true><<<dim3(((ncb + 3) / 4) * (D / 64), ncb, B), 256, 0, st>>>(dy, S, G, D, wfold, nullptr, dx);
  TM_CHECK_LAUNCH();
  ppeg_wgrad_kernel<<<dim3(((ncb + 3) / 4) * (D / 64), (ncb + WRB - 1) / WRB, B), 256, 0, st>>>(x, dy, S, G, D, work);
  TM_CHECK_LAUNCH();
  if (int rc = tm_splitk_reduce(work, dwsum, ppeg_wgrad_slabs(B, G), (long long)D * 50, 1.0f, 0, stream)) return rc;
  ppeg_unfold_kernel<<<(D + 63) / 64, 64, 0, st>>>(dwsum, D, dw7, db7, dw5, db5, dw3, db3);
  TM_CHECK_LAUNCH();
  return 0;
}
