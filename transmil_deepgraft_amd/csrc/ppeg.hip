// PPEG: pyramid positional encoding generator (code/models/TransMIL.py:60-75).
//
//   out = dw7x7(g) + g + dw5x5(g) + dw3x3(g)   on the G x G patch grid, zero padding,
//   per-channel biases; the class token (row 0) passes through.
//
// The three depthwise convolutions, the identity and the three biases fold into
// ONE 7x7 depthwise stencil (w = w7 + pad(w5) + pad(w3) + delta, b = b7+b5+b3),
// applied channel-last directly on the [B, S, D] fp32 residual stream: token
// t = 1 + r*G + c (row-major, :71).  No transpose to NCHW, no padded copy.
// Blocks own a tile of grid cells x 64 channels staged through LDS (one burst of coalesced
// 256-B channel-row loads per window); HBM-bound.
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

// LDS-tiled stencil: a 256-thread block owns a TR x TC tile of grid cells x 64 channels.  The
// (TR + 6) x (TC + 6) input window (zero outside the grid) is requested in one burst of 16-B
// loads (a wave covers 4 cells x 64 channels: four 256-B segments) into LDS [cell][64]; then
// thread (channel, g) computes output rows 2g, 2g + 1 of the tile (16 cells x 49 taps) from LDS
// (consecutive channels in consecutive banks) and stores 256-B channel rows.
// grid (ceil(G / TC) * D / 64, ceil(G / TR), B), block 256.
constexpr int TR = 8, TC = 8, WR = TR + KS - 1, WC = TC + KS - 1;  // 14 x 14 window
constexpr int WIN = WR * WC;                                       // 196 cells
constexpr int TILE_LDS = WIN * 64 * 4;                             // 50 KB

// the block's input window into LDS (zero outside the G x G grid)
TM_DEV void load_window(float* win, const float* __restrict__ xb, int G, int D, int r0, int c0) {
  const int tid = threadIdx.x;
  constexpr int PIECES = WIN * 16;              // 16-B pieces (4 channels each)
  constexpr int PER = (PIECES + 255) / 256;     // 13: every load in flight before the first LDS write
  f32x4 v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = u * 256 + tid, cell = i >> 4, c4 = (i & 15) * 4;
    const int rr = r0 - R + cell / WC, cc = c0 - R + cell % WC;
    v[u] = (i < PIECES && rr >= 0 && rr < G && cc >= 0 && cc < G)
               ? *(const f32x4*)(xb + (size_t)(rr * G + cc) * D + c4) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = u * 256 + tid;
    if (i < PIECES) *(f32x4*)(win + (i >> 4) * 64 + (i & 15) * 4) = v[u];
  }
}

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

template <bool BWD_DATA>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void ppeg_stencil_kernel(const float* __restrict__ x, int S, int G, int D,
                                                           const float* __restrict__ wf, const float* __restrict__ bf,
                                                           float* __restrict__ y, DropPad dp) {
  extern __shared__ __attribute__((aligned(16))) float win[];
  const int nchunk = D / 64;
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int chunk = blockIdx.x % nchunk, ch = chunk * 64 + lane;
  const int r0 = blockIdx.y * TR, c0 = (blockIdx.x / nchunk) * TC, b = blockIdx.z;
  float* yb = y + (size_t)b * S * D;
  const bool fuse = BWD_DATA && dp.out != nullptr;
  const uint64_t seed = fuse && dp.p > 0.f ? effective_seed(dp.seed0, dp.seed_ptr) : 0;
  if (blockIdx.x < (unsigned)nchunk && blockIdx.y == 0) {
    if (g == 0) {  // class token passes through
      const float v = x[(size_t)b * S * D + ch];
      yb[ch] = v;
      if (fuse) droppad_store(dp, seed, b, S, D, 0, ch, v);
    }
    if (fuse)  // the front pad rows of dout are zero
      for (int t = g; t < dp.pad; t += 4) {
        const size_t o = ((size_t)b * dp.n_pad + t) * D + ch;
        if (dp.dtype == TM_BF16) ((bf16*)dp.out)[o] = (bf16)0.f;
        else ((float*)dp.out)[o] = 0.f;
      }
  }
  load_window(win, x + (size_t)b * S * D + D + chunk * 64, G, D, r0, c0);
  float w[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) w[t] = wf[(size_t)(BWD_DATA ? NT - 1 - t : t) * D + ch];
  const float bias = BWD_DATA ? 0.f : bf[ch];
  __syncthreads();
  float acc[2][TC];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TC; ++j) acc[i][j] = bias;
#pragma unroll
  for (int ir = 0; ir < 2 + KS - 1; ++ir) {   // window rows 2g .. 2g + 7
    float xv[WC];
#pragma unroll
    for (int ic = 0; ic < WC; ++ic) xv[ic] = win[((2 * g + ir) * WC + ic) * 64 + lane];
#pragma unroll
    for (int orow = 0; orow < 2; ++orow) {
      const int dy = ir - orow;
      if (dy < 0 || dy >= KS) continue;
#pragma unroll
      for (int oc = 0; oc < TC; ++oc)
#pragma unroll
        for (int dx = 0; dx < KS; ++dx) acc[orow][oc] = fmaf(w[dy * KS + dx], xv[oc + dx], acc[orow][oc]);
    }
  }
#pragma unroll
  for (int orow = 0; orow < 2; ++orow)
#pragma unroll
    for (int oc = 0; oc < TC; ++oc) {
      const int r = r0 + 2 * g + orow, c = c0 + oc;
      if (r < G && c < G) {
        yb[(size_t)(1 + r * G + c) * D + ch] = acc[orow][oc];
        if (fuse) droppad_store(dp, seed, b, S, D, 1 + r * G + c, ch, acc[orow][oc]);
      }
    }
}

// weight / bias gradient partials: dW[ch][tap] = sum_cells dy[cell][ch] x[cell + tap][ch],
// db[ch] = sum_cells dy[cell][ch].  A block walks WT tiles along a row of tiles (x window and dy
// tile through LDS, as the stencil), thread (channel, g) accumulating its 16 cells x 49 taps;
// the 4 g partials are summed in order through LDS.  grid (ceil(nTC / WT) * D / 64, nTR, B),
// partial slab index = (b * gridDim.y + by) * gridDim.x/nchunk + bx/nchunk, layout [slab][ch][50].
constexpr int WT_DEFAULT = 3;   // G = 91: 4 column groups x 12 row tiles x 8 channel chunks = 384 blocks (scripts/dev/ppeg_wt.py: 43.0 vs 48.3 us at 4)
#ifdef TM_DIAG
int g_ppeg_wt = 0;   // diagnostic build: tiles per wgrad block (0: WT_DEFAULT)
#define PPEG_WT (g_ppeg_wt > 0 ? g_ppeg_wt : WT_DEFAULT)
#else
#define PPEG_WT WT_DEFAULT
#endif
constexpr int DY_LDS = TR * TC * 64 * 4;   // 16 KB
__global__ __launch_bounds__(256) void ppeg_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy_,
                                                         int S, int G, int D, int WT, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float win[];
  float* dyt = win + WIN * 64;
  const int nchunk = D / 64;
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int chunk = blockIdx.x % nchunk;
  const int r0 = blockIdx.y * TR, b = blockIdx.z;
  const int ntc = (G + TC - 1) / TC;
  const float* xb = x + (size_t)b * S * D + D + chunk * 64;
  const float* gb = dy_ + (size_t)b * S * D + D + chunk * 64;
  float acc[NT + 1];
#pragma unroll
  for (int t = 0; t <= NT; ++t) acc[t] = 0.f;
  for (int tcol = (blockIdx.x / nchunk) * WT; tcol < min(ntc, (int)(blockIdx.x / nchunk) * WT + WT); ++tcol) {
    const int c0 = tcol * TC;
    __syncthreads();  // previous tile's LDS reads done
    load_window(win, xb, G, D, r0, c0);
    for (int i = tid; i < TR * TC * 16; i += 256) {
      const int cell = i >> 4, c4 = (i & 15) * 4, rr = r0 + cell / TC, cc = c0 + cell % TC;
      *(f32x4*)(dyt + cell * 64 + c4) = (rr < G && cc < G) ? *(const f32x4*)(gb + (size_t)(rr * G + cc) * D + c4)
                                                            : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
#pragma unroll
    for (int orow = 0; orow < 2; ++orow) {
      const int tr = 2 * g + orow;
      float gv[TC];
#pragma unroll
      for (int oc = 0; oc < TC; ++oc) {
        gv[oc] = dyt[(tr * TC + oc) * 64 + lane];
        acc[NT] += gv[oc];
      }
#pragma unroll
      for (int dy = 0; dy < KS; ++dy) {
        float xv[WC];
#pragma unroll
        for (int ic = 0; ic < WC; ++ic) xv[ic] = win[((tr + dy) * WC + ic) * 64 + lane];
#pragma unroll
        for (int oc = 0; oc < TC; ++oc)
#pragma unroll
          for (int dx = 0; dx < KS; ++dx) acc[dy * KS + dx] = fmaf(gv[oc], xv[oc + dx], acc[dy * KS + dx]);
      }
    }
  }
  __syncthreads();
  float* red = win;  // [4][64][NT + 1]
#pragma unroll
  for (int t = 0; t <= NT; ++t) red[(g * 64 + lane) * (NT + 1) + t] = acc[t];
  __syncthreads();
  const int slab = (b * gridDim.y + blockIdx.y) * (gridDim.x / nchunk) + blockIdx.x / nchunk;
  float* dst = part + (size_t)slab * D * (NT + 1) + (size_t)chunk * 64 * (NT + 1);
  for (int e = tid; e < 64 * (NT + 1); e += 256)
    dst[e] = (red[e] + red[64 * (NT + 1) + e]) + (red[2 * 64 * (NT + 1) + e] + red[3 * 64 * (NT + 1) + e]);
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

#ifdef TM_DIAG
extern "C" void tm_debug_set_ppeg_wt(int v) { g_ppeg_wt = v; }
#endif

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
  const dim3 grid(((G + TC - 1) / TC) * (D / 64), (G + TR - 1) / TR, B);
  ppeg_stencil_kernel<false><<<grid, 256, TILE_LDS, (hipStream_t)stream>>>(x, 1 + G * G, G, D, wfold, bfold, y,
                                                                          DropPad{});
  TM_CHECK_LAUNCH();
  return 0;
}

static dim3 wgrad_grid(int B, int G, int D, int wt) {
  const int ntc = (G + TC - 1) / TC;
  return dim3(((ntc + wt - 1) / wt) * (D / 64), (G + TR - 1) / TR, B);
}

static int ppeg_wgrad_slabs(int B, int G, int wt) {
  const dim3 g = wgrad_grid(B, G, 64, wt);
  return (int)(g.x * g.y * g.z);
}

extern "C" long long tm_ppeg_bwd_workspace(int B, int G, int D) {
#ifdef TM_DIAG
  const int wt = 1;   // the largest slab count any diagnostic WT needs
#else
  const int wt = PPEG_WT;
#endif
  return (long long)ppeg_wgrad_slabs(B, G, wt) * D * 50 * (long long)sizeof(float);
}

// dy: [B,S,D] upstream gradient; x: PPEG input.  dx written (=); weight grads written.
extern "C" int tm_ppeg_bwd(const float* x, const float* dy, int B, int G, int D, const float* wfold, float* dx,
                           float* work, float* dwsum, float* dw7, float* db7, float* dw5, float* db5, float* dw3,
                           float* db3, int dtype, void* dout, int n_pad, int pad, float p, uint64_t seed,
                           const uint64_t* seed_ptr, void* stream) {
  TM_REQUIRE(x && dy && dx && dx != dy && D % 64 == 0, "ppeg_bwd: bad args");
  TM_REQUIRE(!dout || ((dtype == TM_BF16 || dtype == TM_F32) && n_pad >= pad + 1 + G * G && pad >= 0),
             "ppeg_bwd: bad dropout-pad output");
  hipStream_t st = (hipStream_t)stream;
  const int S = 1 + G * G;
  const DropPad dp{dout, dtype, n_pad, pad, p, p > 0.f ? 1.f / (1.f - p) : 1.f, seed, seed_ptr};
  ppeg_stencil_kernel<true><<<dim3(((G + TC - 1) / TC) * (D / 64), (G + TR - 1) / TR, B), 256, TILE_LDS, st>>>(
      dy, S, G, D, wfold, nullptr, dx, dp);
  TM_CHECK_LAUNCH();
  tm_allow_smem(ppeg_wgrad_kernel, TILE_LDS + DY_LDS);
  const int wt = PPEG_WT;
  ppeg_wgrad_kernel<<<wgrad_grid(B, G, D, wt), 256, TILE_LDS + DY_LDS, st>>>(x, dy, S, G, D, wt, work);
  TM_CHECK_LAUNCH();
  (void)dwsum;
  ppeg_wgrad_reduce_kernel<<<(D * (NT + 1) + 255) / 256, 256, 0, st>>>(work, ppeg_wgrad_slabs(B, G, wt), D, dw7, db7, dw5,
                                                                     db5, dw3, db3);
  TM_CHECK_LAUNCH();
  return 0;
}
