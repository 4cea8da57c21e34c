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
// Persistent tile walkers (the step's PPEG launches).  The tiles of one 64-channel chunk belong to
// a team of workgroups launched as blockIdx.x = chunk + nchunk * team, so with the round-robin
// dispatch a chunk's team sits on ONE XCD (nchunk = 8): the 3-cell halo each 8 x 8 tile re-reads is
// served by that XCD's L2 (the chunk's slice of a [B, S, 512] tensor is 2.1 MB).  A member walks
// tiles team, team + nteam, ... (row-major: the team works on neighbouring tiles at the same time)
// and requests the next tile's operands into registers before it computes the current one, so the
// HBM / L2 round trip overlaps the arithmetic.
//
// Register blocking: a thread owns 4 channels (one 16-B LDS piece) and 4 cells, so one ds_read_b128
// feeds 4 FMAs per tap it meets (the one-channel-per-lane form was LDS-instruction bound:
// 0.38 ds_read_b32 per FMA against the ~0.25 the VALU rate allows).
//   stencil (forward y = conv(x) + b; backward dx = conv_flipped(dy) + the fused dropout-pad store):
//     256 threads = 16 channel quads x 2 column halves x 8 tile rows; per window row dy: 10 x-pieces
//     + 7 tap pieces -> 4 cells x 7 taps x 4 channels (the same tap order as before: window rows,
//     then columns).
//   weight gradient dW[tap] += dy(cell) x(cell + tap - 3), db += dy(cell): 224 threads = 16 channel
//     quads x 7 tap rows x 2 tile-row halves (+ 32 threads for db): per tile row, the dy row (8
//     pieces) and the x window row (14 pieces) -> 7 taps x 8 cells x 4 channels, accumulated in
//     registers over the member's tiles, then ONE [D][50] partial slab per member.
constexpr int ST_THREADS = 256;
constexpr int ST_PER = (WIN * 16 + ST_THREADS - 1) / ST_THREADS;   // 16-B window pieces per thread: 13
constexpr int TAPS_LDS = NT * 64 * 4;                               // the chunk's folded taps: 12.25 KB
constexpr int ST_LDS = TILE_LDS + TAPS_LDS;                         // 61.25 KB: two workgroups per CU
constexpr int DYT_LDS = TR * TC * 64 * 4;                           // dy tile: 16 KB
constexpr int WG_LDS = TILE_LDS + DYT_LDS;                          // 65 KB
constexpr int DYT_PER = TR * TC * 16 / ST_THREADS;                  // 4

// tiles per team member for a chunk of `ntiles` tiles and at most `cap` members: the balanced team size
inline int walk_team(int ntiles, int cap) {
  cap = cap < 1 ? 1 : cap;
  const int per = (ntiles + cap - 1) / cap;
  return (ntiles + per - 1) / per;
}

TM_DEV f32x4 ld4(const float* p) { return *(const f32x4*)p; }

// the window of tile t (zero outside the grid): piece i = cell i / 16, channel quad i % 16
// (rsrc: the bag's G x G cells from `base`, bounds-checked: out-of-grid pieces read zeros)
template <int PER>
TM_DEV void fetch_window(f32x4 (&v)[PER], __amdgpu_buffer_rsrc_t rsrc, int t, int ntc, int G, int D, int tid) {
  const int r0 = (t / ntc) * TR, c0 = (t % ntc) * TC;
  const int c4 = (tid & 15) * 4;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int cell = u * (ST_THREADS / 16) + (tid >> 4);
    const int rr = r0 - R + cell / WC, cc = c0 - R + cell % WC;
    const bool in = (cell < WIN) & ((unsigned)rr < (unsigned)G) & ((unsigned)cc < (unsigned)G);
    v[u] = tm_bload4(rsrc, in ? (unsigned)((rr * G + cc) * D + c4) * 4u : TM_OOB);
  }
}
template <int PER>
TM_DEV void stage_window(float* win, const f32x4 (&v)[PER], int tid) {
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = u * ST_THREADS + tid;
    if (i < WIN * 16) *(f32x4*)(win + (i >> 4) * 64 + (i & 15) * 4) = v[u];
  }
}

// 4 consecutive channels of droppad_store as one 8-B (bf16) / 16-B (fp32) store
TM_DEV void droppad_store4(const DropPad& dp, uint64_t seed, int b, int S, int D, int t, int ch0, f32x4 v) {
  if (dp.p > 0.f) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = dropout_u01(seed, (uint32_t)(b * S + t), (uint32_t)(ch0 + e)) >= dp.p ? v[e] * dp.scale : 0.f;
  }
  const size_t o = ((size_t)b * dp.n_pad + dp.pad + t) * D + ch0;
  if (dp.dtype == TM_BF16) *(bf16x4*)((bf16*)dp.out + o) = (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  else *(f32x4*)((float*)dp.out + o) = v;
}

template <bool BWD>
__global__ __launch_bounds__(ST_THREADS) void ppeg_stencil_walk_kernel(const float* __restrict__ src, int S, int G,
                                                                      int D, int nteam, const float* __restrict__ wf,
                                                                      const float* __restrict__ bf,
                                                                      float* __restrict__ y, DropPad dp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* win = lds;                  // [WIN][64]: x (forward) / dy (backward)
  float* wl = lds + WIN * 64;        // [49][64] taps (flipped for the backward)
  const int nchunk = D / 64;
  const int tid = threadIdx.x, cq = tid & 15, hf = (tid >> 4) & 1, orow = tid >> 5;
  const int chunk = blockIdx.x % nchunk, team = blockIdx.x / nchunk, b = blockIdx.y;
  const int ch0 = chunk * 64 + 4 * cq;
  const int ntc = (G + TC - 1) / TC, ntiles = ((G + TR - 1) / TR) * ntc;
  const float* sb = src + (size_t)b * S * D + D + chunk * 64;
  float* yb = y + (size_t)b * S * D;
  const bool fuse = BWD && dp.out != nullptr;
  const uint64_t seed = fuse && dp.p > 0.f ? effective_seed(dp.seed0, dp.seed_ptr) : 0;
  if (team == 0) {
    const int lane = tid & 63, wv = tid >> 6, ch = chunk * 64 + lane;
    if (wv == 0) {  // the class token passes through
      const float v = src[(size_t)b * S * D + ch];
      yb[ch] = v;
      if (fuse) droppad_store(dp, seed, b, S, D, 0, ch, v);
    }
    if (fuse)      // the front pad rows of dout are zero
      for (int t = wv; t < dp.pad; t += ST_THREADS / 64) {
        const size_t o = ((size_t)b * dp.n_pad + t) * D + ch;
        if (dp.dtype == TM_BF16) ((bf16*)dp.out)[o] = (bf16)0.f;
        else ((float*)dp.out)[o] = 0.f;
      }
  }
  for (int i = tid; i < NT * 16; i += ST_THREADS) {
    const int t = i >> 4, q = (i & 15) * 4;
    *(f32x4*)(wl + t * 64 + q) = ld4(wf + (size_t)(BWD ? NT - 1 - t : t) * D + chunk * 64 + q);
  }
  const f32x4 bias = BWD ? (f32x4){0.f, 0.f, 0.f, 0.f} : ld4(bf + ch0);
  const __amdgpu_buffer_rsrc_t rs = tm_rsrc(sb, (unsigned)(G * G * D) * 4u);
  f32x4 pa[ST_PER];
  if (team < ntiles) fetch_window(pa, rs, team, ntc, G, D, tid);
  for (int t = team; t < ntiles; t += nteam) {
    __syncthreads();   // the previous tile's LDS reads are done (first pass: the taps are written)
    stage_window(win, pa, tid);
    __syncthreads();
    if (t + nteam < ntiles) fetch_window(pa, rs, t + nteam, ntc, G, D, tid);   // in flight meanwhile
    const int r0 = (t / ntc) * TR, c0 = (t % ntc) * TC;
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bias;
#pragma unroll 1
    for (int dy = 0; dy < KS; ++dy) {
      const float* wr = win + ((orow + dy) * WC + 4 * hf) * 64 + 4 * cq;
      f32x4 xv[4 + KS - 1], wt[KS];
#pragma unroll
      for (int ic = 0; ic < 4 + KS - 1; ++ic) xv[ic] = ld4(wr + ic * 64);
#pragma unroll
      for (int dx = 0; dx < KS; ++dx) wt[dx] = ld4(wl + (dy * KS + dx) * 64 + 4 * cq);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int dx = 0; dx < KS; ++dx)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[j][e] = fmaf(wt[dx][e], xv[j + dx][e], acc[j][e]);
    }
    const int r = r0 + orow;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 4 * hf + j;
      if (r < G && c < G) {
        const int tok = 1 + r * G + c;
        *(f32x4*)(yb + (size_t)tok * D + ch0) = acc[j];
        if (fuse) droppad_store4(dp, seed, b, S, D, tok, ch0, acc[j]);
      }
    }
  }
}

__global__ __launch_bounds__(ST_THREADS) void ppeg_wgrad_walk_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ dy_, int S, int G, int D,
                                                                    int nteam, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* win = lds;                  // [WIN][64] x window
  float* dyt = lds + WIN * 64;       // [TR * TC][64] dy tile
  const int nchunk = D / 64;
  const int tid = threadIdx.x, cq = tid & 15, g = tid >> 4;   // g < 14: tap row g >> 1, tile rows 4 (g & 1) ..
  const int chunk = blockIdx.x % nchunk, team = blockIdx.x / nchunk, b = blockIdx.y;
  const int ntc = (G + TC - 1) / TC, ntiles = ((G + TR - 1) / TR) * ntc;
  const float* xb = x + (size_t)b * S * D + D + chunk * 64;
  const float* gb = dy_ + (size_t)b * S * D + D + chunk * 64;
  const int tdy = g >> 1, rs = g & 1;   // g = 14 / 15: the bias sums of tile rows 0-3 / 4-7
  f32x4 accw[KS];
#pragma unroll
  for (int dx = 0; dx < KS; ++dx) accw[dx] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rx = tm_rsrc(xb, (unsigned)(G * G * D) * 4u), rg = tm_rsrc(gb, (unsigned)(G * G * D) * 4u);
  f32x4 px[ST_PER], pg[DYT_PER];
  auto fetch = [&](int t) {
    fetch_window(px, rx, t, ntc, G, D, tid);
    const int r0 = (t / ntc) * TR, c0 = (t % ntc) * TC;
#pragma unroll
    for (int u = 0; u < DYT_PER; ++u) {
      const int i = u * ST_THREADS + tid, cell = i >> 4, c4 = (i & 15) * 4;
      const int rr = r0 + cell / TC, cc = c0 + cell % TC;
      pg[u] = tm_bload4(rg, ((rr < G) & (cc < G)) ? (unsigned)((rr * G + cc) * D + c4) * 4u : TM_OOB);
    }
  };
  if (team < ntiles) fetch(team);
  for (int t = team; t < ntiles; t += nteam) {
    __syncthreads();
    stage_window(win, px, tid);
#pragma unroll
    for (int u = 0; u < DYT_PER; ++u) {
      const int i = u * ST_THREADS + tid;
      *(f32x4*)(dyt + (i >> 4) * 64 + (i & 15) * 4) = pg[u];
    }
    __syncthreads();
    if (t + nteam < ntiles) fetch(t + nteam);
    if (g < 14) {
#pragma unroll 1
      for (int orow = 4 * rs; orow < 4 * rs + 4; ++orow) {
        f32x4 gv[TC], xv[WC];
#pragma unroll
        for (int j = 0; j < TC; ++j) gv[j] = ld4(dyt + (orow * TC + j) * 64 + 4 * cq);
#pragma unroll
        for (int ic = 0; ic < WC; ++ic) xv[ic] = ld4(win + ((orow + tdy) * WC + ic) * 64 + 4 * cq);
#pragma unroll
        for (int j = 0; j < TC; ++j)
#pragma unroll
          for (int dx = 0; dx < KS; ++dx)
#pragma unroll
            for (int e = 0; e < 4; ++e) accw[dx][e] = fmaf(gv[j][e], xv[j + dx][e], accw[dx][e]);
      }
    } else {
#pragma unroll
      for (int cell = 32 * rs; cell < 32 * rs + 32; ++cell) accw[0] += ld4(dyt + cell * 64 + 4 * cq);
    }
  }
  // partial slab [D][50] of this member: the two tile-row halves summed (rs 0 + rs 1) through LDS
  __syncthreads();
  float* red = lds;   // [2][16 quads][8 rows: 7 tap rows + bias][7][4]
  {
    const int trow = g < 14 ? tdy : 7;
    float* o = red + (((size_t)rs * 16 + cq) * 8 + trow) * 28;
#pragma unroll
    for (int dx = 0; dx < KS; ++dx) *(f32x4*)(o + dx * 4) = accw[dx];
  }
  __syncthreads();
  float* dst = part + ((size_t)b * nteam + team) * D * (NT + 1) + (size_t)chunk * 64 * (NT + 1);
  for (int e = tid; e < 64 * (NT + 1); e += ST_THREADS) {
    const int cl = e / (NT + 1), tp = e - cl * (NT + 1);          // channel of the chunk, tap (49 = bias)
    const int q = cl >> 2, ce = cl & 3;
    const int trow = tp == NT ? 7 : tp / KS, dx = tp == NT ? 0 : tp - (tp / KS) * KS;
    const size_t i0 = (((size_t)0 * 16 + q) * 8 + trow) * 28 + dx * 4 + ce;
    const size_t i1 = (((size_t)1 * 16 + q) * 8 + trow) * 28 + dx * 4 + ce;
    dst[e] = red[i0] + red[i1];
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
// team members per chunk: two 61-65 KB workgroups per CU
static int walk_nteam(int G, int D) {
  const int ntiles = ((G + TR - 1) / TR) * ((G + TC - 1) / TC);
  return walk_team(ntiles, 2 * tm_cu_count() / (D / 64));
}

// x, y: [B, S, D] fp32 with S = 1 + G*G.  y must not alias x.
extern "C" int tm_ppeg_fwd(const float* x, int B, int G, int D, const float* wfold, const float* bfold, float* y,
                           void* stream) {
  TM_REQUIRE(x && y && x != y && D % 64 == 0 && G > 0 && B > 0, "ppeg_fwd: bad args");
  const int nteam = walk_nteam(G, D);
  ppeg_stencil_walk_kernel<false><<<dim3(nteam * (D / 64), B), ST_THREADS, ST_LDS, (hipStream_t)stream>>>(
      x, 1 + G * G, G, D, nteam, wfold, bfold, y, DropPad{});
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_ppeg_bwd_workspace(int B, int G, int D) {
  return (long long)B * walk_nteam(G, D) * D * (NT + 1) * (long long)sizeof(float);
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
  const int nteam = walk_nteam(G, D);
  const dim3 grid(nteam * (D / 64), B);
  ppeg_stencil_walk_kernel<true><<<grid, ST_THREADS, ST_LDS, st>>>(dy, S, G, D, nteam, wfold, nullptr, dx, dp);
  TM_CHECK_LAUNCH();
  tm_allow_smem(ppeg_wgrad_walk_kernel, WG_LDS);
  ppeg_wgrad_walk_kernel<<<grid, ST_THREADS, WG_LDS, st>>>(x, dy, S, G, D, nteam, work);
  TM_CHECK_LAUNCH();
  (void)dwsum;
  ppeg_wgrad_reduce_kernel<<<(D * (NT + 1) + 255) / 256, 256, 0, st>>>(work, B * nteam, D, dw7, db7, dw5, db5, dw3,
                                                                     db3);
  TM_CHECK_LAUNCH();
  return 0;
}
