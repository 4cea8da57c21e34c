// PPEG: pyramid positional encoding generator (code/models/TransMIL.py:60-75).
//
//   out = dw7x7(g) + g + dw5x5(g) + dw3x3(g)   on the G x G patch grid, zero padding,
//   per-channel biases; the class token (row 0) passes through.
//
// The three depthwise convolutions, the identity and the three biases fold into
// ONE 7x7 depthwise stencil (w = w7 + pad(w5) + pad(w3) + delta, b = b7+b5+b3),
// applied channel-last directly on the [B, S, D] fp32 residual stream: token
// t = 1 + r*G + c (row-major, :71).  No transpose to NCHW, no padded copy.
// Persistent workgroups walk tiles of grid cells x 64 channels staged through LDS (coalesced
// 256-B channel-row loads, the next tile's window in flight during the current tile); HBM-bound.
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

// Tiles: TR x TC grid cells x 64 channels; the (TR + 6) x (TC + 6) input window (zero outside
// the grid) sits in LDS as [cell][64] fp32 (consecutive channels in consecutive banks), requested
// as 16-B pieces (a wave covers 4 cells x 64 channels: four 256-B segments).
constexpr int TR = 8, TC = 8, WR = TR + KS - 1, WC = TC + KS - 1;  // 14 x 14 window
constexpr int WIN = WR * WC;                                       // 196 cells
constexpr int TILE_LDS = WIN * 64 * 4;                             // 50 KB

// Backward only, optional: the next layer-backward's first step fused into the stencil's stores --
// dout[b][pad + t][c] = T(keep(b*S + t, c) * scale * dx[b*S + t][c]) and zero pad rows, the
// padded to_out-dropout gradient of the TransLayer below (as tm_dropout_bwd_pad).
struct DropPad {
  void* out;        // null: off
  int dtype, n_pad, pad;
  float p, scale;
  uint64_t seed0;
  const uint64_t* seed_ptr;
};

TM_DEV void droppad_store(const DropPad& dp, uint64_t seed, int b, int S, int D, int t, int ch, float v) {
  if (dp.p > 0.f) v = dropout_u01(seed, (uint32_t)(b * S + t), (uint32_t)ch) >= dp.p ? v * dp.scale : 0.f;
  const size_t o = ((size_t)b * dp.n_pad + dp.pad + t) * D + ch;
  if (dp.dtype == TM_BF16) ((bf16*)dp.out)[o] = (bf16)v;
  else ((float*)dp.out)[o] = v;
}

// ---------------------------------------------------------------------------
// Persistent tile walker (the step's PPEG launches).  The tiles of one 64-channel chunk belong to a
// team of workgroups launched as blockIdx.x = chunk + nchunk * team, so with the round-robin
// dispatch a chunk's team sits on ONE XCD (nchunk = 8): the 3-cell halo every 8 x 8 tile re-reads is
// served by that XCD's L2 (the chunk's x / dy slices are 2.1 MB each).  A team member walks tiles
// team, team + nteam, ... (row-major: the team works on neighbouring tiles at the same time), and
// the next tile's window is requested into registers before the current tile is computed, so its
// HBM / L2 round trip overlaps the stencil arithmetic.  512 threads: wave w computes row w of the
// tile (8 cells x 49 taps per lane = channel), in a fixed tap order (window rows, then
// columns).  BWD: the window of dy gives dx (flipped taps, + the fused dropout-pad store of the layer
// below) and, with the x window beside it, the 49 tap + bias gradient partials of the tile's cells
// (dW[tap] += dy[cell] x[cell + tap - 3]), kept in registers over the member's tiles and summed over
// its 8 waves in a fixed order into ONE [D][50] partial slab per member (the x / dy windows are read
// once; the separate weight-gradient pass and its second read of dy / x are gone).
constexpr int WALK_THREADS = 512;
constexpr int WALK_PER = (WIN * 16 + WALK_THREADS - 1) / WALK_THREADS;   // 16-B window pieces per thread: 7
constexpr int WALK_RED = 8 * 64 * (NT + 1) * 4;                          // 102 KB: the 8 waves' partials

constexpr int WALK_W = NT * 64 * 4;                                      // the chunk's folded taps: 12.25 KB
template <bool BWD>
constexpr int walk_lds() { return (BWD ? (2 * TILE_LDS > WALK_RED ? 2 * TILE_LDS : WALK_RED) : TILE_LDS) + WALK_W; }

// tiles per team member for a chunk of `ntiles` tiles and at most `cap` members: the balanced team size
inline int walk_team(int ntiles, int cap) {
  cap = cap < 1 ? 1 : cap;
  const int per = (ntiles + cap - 1) / cap;
  return (ntiles + per - 1) / per;
}

template <bool BWD>
__global__ __launch_bounds__(WALK_THREADS) void ppeg_walk_kernel(const float* __restrict__ src,
                                                                 const float* __restrict__ xw, int S, int G, int D,
                                                                 int nteam, const float* __restrict__ wf,
                                                                 const float* __restrict__ bf, float* __restrict__ y,
                                                                 DropPad dp, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* win = lds;                        // [WIN][64]: x (forward) / dy (backward)
  float* winx = lds + WIN * 64;            // backward: the x window
  float* wl = lds + (walk_lds<BWD>() - WALK_W) / 4;   // [49][64] taps (flipped for the backward)
  const int nchunk = D / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int chunk = blockIdx.x % nchunk, team = blockIdx.x / nchunk, b = blockIdx.y;
  const int ch = chunk * 64 + lane;
  const int ntc = (G + TC - 1) / TC, ntiles = ((G + TR - 1) / TR) * ntc;
  const float* sb = src + (size_t)b * S * D + D + chunk * 64;
  const float* xb = BWD ? xw + (size_t)b * S * D + D + chunk * 64 : nullptr;
  float* yb = y + (size_t)b * S * D;
  const bool fuse = BWD && dp.out != nullptr;
  const uint64_t seed = fuse && dp.p > 0.f ? effective_seed(dp.seed0, dp.seed_ptr) : 0;
  if (team == 0) {
    if (w == 0) {  // the class token passes through
      const float v = src[(size_t)b * S * D + ch];
      yb[ch] = v;
      if (fuse) droppad_store(dp, seed, b, S, D, 0, ch, v);
    }
    if (fuse)      // the front pad rows of dout are zero
      for (int t = w; t < dp.pad; t += WALK_THREADS / 64) {
        const size_t o = ((size_t)b * dp.n_pad + t) * D + ch;
        if (dp.dtype == TM_BF16) ((bf16*)dp.out)[o] = (bf16)0.f;
        else ((float*)dp.out)[o] = 0.f;
      }
  }
  for (int t = w; t < NT; t += WALK_THREADS / 64) wl[t * 64 + lane] = wf[(size_t)(BWD ? NT - 1 - t : t) * D + ch];
  const float bias = BWD ? 0.f : bf[ch];
  float accw[BWD ? NT + 1 : 1];
#pragma unroll
  for (int t = 0; t < (BWD ? NT + 1 : 1); ++t) accw[t] = 0.f;

  // window pieces of tile t (zero outside the grid): piece i = cell i / 16, channels 4 (i % 16)
  f32x4 pa[WALK_PER], pb[BWD ? WALK_PER : 1];
  auto fetch = [&](int t) {
    const int r0 = (t / ntc) * TR, c0 = (t % ntc) * TC;
#pragma unroll
    for (int u = 0; u < WALK_PER; ++u) {
      const int i = u * WALK_THREADS + tid, cell = i >> 4, c4 = (i & 15) * 4;
      const int rr = r0 - R + cell / WC, cc = c0 - R + cell % WC;
      const bool in = i < WIN * 16 && rr >= 0 && rr < G && cc >= 0 && cc < G;
      const size_t o = (size_t)(rr * G + cc) * D + c4;
      pa[u] = in ? *(const f32x4*)(sb + o) : (f32x4){0.f, 0.f, 0.f, 0.f};
      if constexpr (BWD) pb[u] = in ? *(const f32x4*)(xb + o) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int u = 0; u < WALK_PER; ++u) {
      const int i = u * WALK_THREADS + tid;
      if (i < WIN * 16) {
        *(f32x4*)(win + (i >> 4) * 64 + (i & 15) * 4) = pa[u];
        if constexpr (BWD) *(f32x4*)(winx + (i >> 4) * 64 + (i & 15) * 4) = pb[u];
      }
    }
  };
  if (team < ntiles) fetch(team);
  for (int t = team; t < ntiles; t += nteam) {
    __syncthreads();   // the previous tile's LDS reads are done
    stage();
    __syncthreads();
    if (t + nteam < ntiles) fetch(t + nteam);   // in flight through this tile's arithmetic
    const int r0 = (t / ntc) * TR, c0 = (t % ntc) * TC;
    float acc[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) acc[j] = bias;
#pragma unroll 1
    for (int dy = 0; dy < KS; ++dy) {   // window row w + dy (rolled: the row's 14 + 7 values live at once)
      float xv[WC], wt[KS];
#pragma unroll
      for (int ic = 0; ic < WC; ++ic) xv[ic] = win[((w + dy) * WC + ic) * 64 + lane];
#pragma unroll
      for (int dx = 0; dx < KS; ++dx) wt[dx] = wl[(dy * KS + dx) * 64 + lane];
#pragma unroll
      for (int oc = 0; oc < TC; ++oc)
#pragma unroll
        for (int dx = 0; dx < KS; ++dx) acc[oc] = fmaf(wt[dx], xv[oc + dx], acc[oc]);
    }
    const int r = r0 + w;
#pragma unroll
    for (int oc = 0; oc < TC; ++oc) {
      const int c = c0 + oc;
      if (r < G && c < G) {
        yb[(size_t)(1 + r * G + c) * D + ch] = acc[oc];
        if (fuse) droppad_store(dp, seed, b, S, D, 1 + r * G + c, ch, acc[oc]);
      }
    }
    if constexpr (BWD) {
      // dW[dy][dx] += dy(r, c) x(r + dy - 3, c + dx - 3): dy(r, c) = centre of the dy window
      float gv[TC];
#pragma unroll
      for (int oc = 0; oc < TC; ++oc) {
        gv[oc] = win[((w + R) * WC + oc + R) * 64 + lane];
        accw[NT] += gv[oc];
      }
#pragma unroll
      for (int dy = 0; dy < KS; ++dy) {   // unrolled: accw is indexed by dy at compile time
        float xv[WC];
#pragma unroll
        for (int ic = 0; ic < WC; ++ic) xv[ic] = winx[((w + dy) * WC + ic) * 64 + lane];
#pragma unroll
        for (int oc = 0; oc < TC; ++oc)
#pragma unroll
          for (int dx = 0; dx < KS; ++dx) accw[dy * KS + dx] = fmaf(gv[oc], xv[oc + dx], accw[dy * KS + dx]);
      }
    }
  }
  if constexpr (BWD) {
    __syncthreads();   // the windows are no longer read: the LDS takes the 8 waves' partials
    float* red = lds;  // [8][64][NT + 1]
#pragma unroll
    for (int t = 0; t <= NT; ++t) red[(w * 64 + lane) * (NT + 1) + t] = accw[t];
    __syncthreads();
    float* dst = part + ((size_t)b * nteam + team) * D * (NT + 1) + (size_t)chunk * 64 * (NT + 1);
    constexpr int E = 64 * (NT + 1);
    for (int e = tid; e < E; e += WALK_THREADS) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) s += red[v * E + e];
      dst[e] = s;
    }
  }
}

// unfold folded gradients: dw7 = dwf, dw5 = centre 5x5, dw3 = centre 3x3, db* = db
// the weight-gradient partial slabs summed (in slab order, as tm_splitk_reduce) straight into the
// unfolded gradients: thread i = (ch, t) of the [D][50] partial layout, t < 49 a tap of the folded
// 7x7 kernel (its 5x5 / 3x3 centre taps also feed dw5 / dw3: the fold is a sum), t = 49 the bias
__global__ __launch_bounds__(256) void ppeg_wgrad_reduce_kernel(const float* __restrict__ part, int slabs, int D,
                                                                float* __restrict__ dw7, float* __restrict__ db7,
                                                                float* __restrict__ dw5, float* __restrict__ db5,
                                                                float* __restrict__ dw3, float* __restrict__ db3) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const size_t count = (size_t)D * (NT + 1);
  if (i >= (int)count) return;
  constexpr int U = 12;
  float s = 0.f;
  for (int z0 = 0; z0 < slabs; z0 += U) {
    float v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = part[(size_t)min(z0 + k, slabs - 1) * count + i];
#pragma unroll
    for (int k = 0; k < U; ++k) s += z0 + k < slabs ? v[k] : 0.f;
  }
  const int ch = i / (NT + 1), t = i - ch * (NT + 1);
  if (t == NT) { db7[ch] = s; db5[ch] = s; db3[ch] = s; return; }
  dw7[(size_t)ch * NT + t] = s;
  const int dy = t / KS, dx = t - dy * KS;
  if (dy >= 1 && dy <= 5 && dx >= 1 && dx <= 5) dw5[(size_t)ch * 25 + (dy - 1) * 5 + dx - 1] = s;
  if (dy >= 2 && dy <= 4 && dx >= 2 && dx <= 4) dw3[(size_t)ch * 9 + (dy - 2) * 3 + dx - 2] = s;
}

}  // namespace


extern "C" int tm_ppeg_fold(const float* w7, const float* b7, const float* w5, const float* b5, const float* w3,
                            const float* b3, int D, float* wfold, float* bfold, void* stream) {
  ppeg_fold_kernel<<<(D + 63) / 64, 64, 0, (hipStream_t)stream>>>(w7, b7, w5, b5, w3, b3, D, wfold, bfold);
  TM_CHECK_LAUNCH();
  return 0;
}

// x, y: [B, S, D] fp32 with S = 1 + G*G.  y must not alias x.
// team members of the walker per chunk: the forward (50 KB of LDS) two workgroups per CU, the
// backward (100 KB) one
static int walk_nteam(int G, int D, bool bwd) {
  const int ntiles = ((G + TR - 1) / TR) * ((G + TC - 1) / TC);
  const int nchunk = D / 64;
  return walk_team(ntiles, (bwd ? 1 : 2) * tm_cu_count() / nchunk);
}

// x, y: [B, S, D] fp32 with S = 1 + G*G.  y must not alias x.
extern "C" int tm_ppeg_fwd(const float* x, int B, int G, int D, const float* wfold, const float* bfold, float* y,
                           void* stream) {
  TM_REQUIRE(x && y && x != y && D % 64 == 0 && G > 0 && B > 0, "ppeg_fwd: bad args");
  const int nteam = walk_nteam(G, D, false);
  tm_allow_smem(ppeg_walk_kernel<false>, walk_lds<false>());
  ppeg_walk_kernel<false><<<dim3(nteam * (D / 64), B), WALK_THREADS, walk_lds<false>(), (hipStream_t)stream>>>(
      x, nullptr, 1 + G * G, G, D, nteam, wfold, bfold, y, DropPad{}, nullptr);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_ppeg_bwd_workspace(int B, int G, int D) {
  return (long long)B * walk_nteam(G, D, true) * D * (NT + 1) * (long long)sizeof(float);
}

// dy: [B,S,D] upstream gradient; x: PPEG input.  dx written (=); weight grads written.
extern "C" int tm_ppeg_bwd(const float* x, const float* dy, int B, int G, int D, const float* wfold, float* dx,
                           float* work, float* dwsum, float* dw7, float* db7, float* dw5, float* db5, float* dw3,
                           float* db3, int dtype, void* dout, int n_pad, int pad, float p, uint64_t seed,
                           const uint64_t* seed_ptr, void* stream) {
  TM_REQUIRE(x && dy && dx && dx != dy && D % 64 == 0 && G > 0 && B > 0, "ppeg_bwd: bad args");
  TM_REQUIRE(!dout || ((dtype == TM_BF16 || dtype == TM_F32) && n_pad >= pad + 1 + G * G && pad >= 0),
             "ppeg_bwd: bad dropout-pad output");
  hipStream_t st = (hipStream_t)stream;
  const int S = 1 + G * G;
  const DropPad dp{dout, dtype, n_pad, pad, p, p > 0.f ? 1.f / (1.f - p) : 1.f, seed, seed_ptr};
  const int nteam = walk_nteam(G, D, true);
  tm_allow_smem(ppeg_walk_kernel<true>, walk_lds<true>());
  ppeg_walk_kernel<true><<<dim3(nteam * (D / 64), B), WALK_THREADS, walk_lds<true>(), st>>>(
      dy, x, S, G, D, nteam, wfold, nullptr, dx, dp, work);
  TM_CHECK_LAUNCH();
  (void)dwsum;
  ppeg_wgrad_reduce_kernel<<<(D * (NT + 1) + 255) / 256, 256, 0, st>>>(work, B * nteam, D, dw7, db7, dw5, db5, dw3,
                                                                     db3);
  TM_CHECK_LAUNCH();
  return 0;
}
