// PPEG: pyramid positional encoding generator (code/models/TransMIL.py:60-75).
//
//   out = dw7x7(g) + g + dw5x5(g) + dw3x3(g)   on the G x G patch grid, zero padding,
//   per-channel biases; the class token (row 0) passes through.
//
// The three depthwise convolutions, the identity and the three biases fold into
// ONE 7x7 depthwise stencil (w = w7 + pad(w5) + pad(w3) + delta, b = b7+b5+b3),
// applied channel-last directly on the [B, S, D] fp32 residual stream: token
// t = 1 + r*G + c (row-major, :71).  No transpose to NCHW, no padded copy.
// Workgroups own tiles of grid cells x 32 channels staged through LDS (coalesced
// 128-B channel-row loads, three workgroups per CU in flight); HBM-bound.
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
// Tile kernels (the step's PPEG launches): one 8 x 8 tile x 32 channels per 256-thread workgroup,
// high occupancy instead of a software pipeline.  The kernels are bound by how many window bytes a
// CU has in flight (one tile's loads, then its arithmetic): 32 channels keep a workgroup's LDS at
// 43-50 KB so three run per CU, and the channel chunk rides in the low bits of blockIdx.x
// (chunk = blockIdx.x % nchunk) so with the round-robin dispatch each XCD serves two chunks and the
// 3-cell halo of neighbouring tiles is re-read from its L2.  Windows sit in LDS with a 48-dword
// (192 B) cell stride: the 16-lane groups of ds_read_b128 then hit 16 distinct 16-B bank slots.
// Register blocking: a thread owns 4 channels (one 16-B piece) and 2 cells, so a ds_read_b128
// feeds 4 FMAs for each tap it meets.
//   stencil (forward y = conv(x) + b; backward dx = conv_flipped(dy) + the fused dropout-pad store):
//     256 threads = 8 channel quads x 4 column pairs x 8 tile rows; per window row: 8 x-pieces +
//     7 tap pieces -> 2 cells x 7 taps x 4 channels, taps in the fixed order window rows, columns.
//   weight gradient dW[tap] += dy(cell) x(cell + tap - 3), db += dy(cell): 224 threads = 8 channel
//     quads x 7 tap rows x 4 tile-row pairs (+ 32 threads for db), WT tiles along a tile row per
//     workgroup, then ONE [D][50] partial slab per workgroup (fixed-order sums).
constexpr int CW = 32;                        // channels per workgroup
constexpr int NQ = CW / 4;                    // channel quads
constexpr int CS = 48;                        // LDS cell stride (dwords)
constexpr int WIN_LDS = WIN * CS * 4;         // 37.6 KB
constexpr int TAP_LDS = NT * NQ * 16;         // 6.1 KB
constexpr int ST_LDS = WIN_LDS + TAP_LDS;     // 43.8 KB: three workgroups per CU
constexpr int DYT_LDS = TR * TC * CS * 4;     // 12 KB
constexpr int WG_LDS = WIN_LDS + DYT_LDS;     // 49.7 KB
constexpr int WIN_PER = (WIN * NQ + 255) / 256;   // 16-B window pieces per thread: 7
constexpr int WT = 3;                         // tiles per weight-gradient workgroup

TM_DEV f32x4 ld4(const float* p) { return *(const f32x4*)p; }

// the 14 x 14 window of the tile at (r0, c0) into LDS (zero outside the grid; rsrc: the bag's G x G
// cells from this chunk's first channel, bounds-checked -> out-of-grid pieces read zeros)
TM_DEV void load_window(float* win, __amdgpu_buffer_rsrc_t rsrc, int r0, int c0, int G, int D, int tid) {
  f32x4 v[WIN_PER];
  const int q4 = (tid & (NQ - 1)) * 4;
#pragma unroll
  for (int u = 0; u < WIN_PER; ++u) {
    const int cell = u * (256 / NQ) + tid / NQ;
    const int rr = r0 - R + cell / WC, cc = c0 - R + cell % WC;
    const bool in = (cell < WIN) & ((unsigned)rr < (unsigned)G) & ((unsigned)cc < (unsigned)G);
    v[u] = tm_bload4(rsrc, in ? (unsigned)((rr * G + cc) * D + q4) * 4u : TM_OOB);
  }
#pragma unroll
  for (int u = 0; u < WIN_PER; ++u) {
    const int cell = u * (256 / NQ) + tid / NQ;
    if (cell < WIN) *(f32x4*)(win + cell * CS + q4) = v[u];
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

// grid (nchunk * ntiles, B), block 256
template <bool BWD>
TM_DEV void ppeg_stencil_body(const float* __restrict__ src, int S, int G, int D, const float* __restrict__ wf,
                              const float* __restrict__ bf, float* __restrict__ y, const DropPad& dp, int bx, int by) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* win = lds;                  // [WIN][CS]: x (forward) / dy (backward)
  float* wl = lds + WIN * CS;        // [49][CW] taps (flipped for the backward)
  const int nchunk = D / CW;
  const int tid = threadIdx.x, cq = tid & (NQ - 1), cp = (tid / NQ) & 3, orow = tid >> 5;
  const int chunk = bx % nchunk, t = bx / nchunk, b = by;
  const int ntc = (G + TC - 1) / TC, r0 = (t / ntc) * TR, c0 = (t % ntc) * TC;
  const int ch0 = chunk * CW + 4 * cq;
  const float* sb = src + (size_t)b * S * D + D + chunk * CW;
  float* yb = y + (size_t)b * S * D;
  const bool fuse = BWD && dp.out != nullptr;
  const uint64_t seed = fuse && dp.p > 0.f ? effective_seed(dp.seed0, dp.seed_ptr) : 0;
  if (t == 0) {
    const int c = chunk * CW + (tid & (CW - 1)), g = tid / CW;
    if (g == 0) {  // the class token passes through
      const float v = src[(size_t)b * S * D + c];
      yb[c] = v;
      if (fuse) droppad_store(dp, seed, b, S, D, 0, c, v);
    }
    if (fuse)      // the front pad rows of dout are zero
      for (int p = g; p < dp.pad; p += 256 / CW) {
        const size_t o = ((size_t)b * dp.n_pad + p) * D + c;
        if (dp.dtype == TM_BF16) ((bf16*)dp.out)[o] = (bf16)0.f;
        else ((float*)dp.out)[o] = 0.f;
      }
  }
  for (int i = tid; i < NT * NQ; i += 256) {
    const int tp = i / NQ, q = (i % NQ) * 4;
    *(f32x4*)(wl + tp * CW + q) = ld4(wf + (size_t)(BWD ? NT - 1 - tp : tp) * D + chunk * CW + q);
  }
  load_window(win, tm_rsrc(sb, (unsigned)(G * G * D) * 4u), r0, c0, G, D, tid);
  const f32x4 bias = BWD ? (f32x4){0.f, 0.f, 0.f, 0.f} : ld4(bf + ch0);
  __syncthreads();
  f32x4 acc[2] = {bias, bias};
#pragma unroll 1
  for (int dy = 0; dy < KS; ++dy) {
    const float* wr = win + ((orow + dy) * WC + 2 * cp) * CS + 4 * cq;
    f32x4 xv[2 + KS - 1], wt[KS];
#pragma unroll
    for (int ic = 0; ic < 2 + KS - 1; ++ic) xv[ic] = ld4(wr + ic * CS);
#pragma unroll
    for (int dx = 0; dx < KS; ++dx) wt[dx] = ld4(wl + (dy * KS + dx) * CW + 4 * cq);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int dx = 0; dx < KS; ++dx)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[j][e] = fmaf(wt[dx][e], xv[j + dx][e], acc[j][e]);
  }
  const int r = r0 + orow;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = c0 + 2 * cp + j;
    if (r < G && c < G) {
      const int tok = 1 + r * G + c;
      *(f32x4*)(yb + (size_t)tok * D + ch0) = acc[j];
      if (fuse) droppad_store4(dp, seed, b, S, D, tok, ch0, acc[j]);
    }
  }
}
template <bool BWD>
__global__ __launch_bounds__(256) void ppeg_stencil_kernel(const float* __restrict__ src, int S, int G, int D,
                                                          const float* __restrict__ wf, const float* __restrict__ bf,
                                                          float* __restrict__ y, DropPad dp) {
  ppeg_stencil_body<BWD>(src, S, G, D, wf, bf, y, dp, blockIdx.x, blockIdx.y);
}

// grid (nchunk * ntr * ceil(ntc / WT), B), block 256; part: Z = B * ntr * ceil(ntc / WT) slabs in four
// regions [Z][D][49], [Z][D][25], [Z][D][9], [Z][D] (see the store loop)
TM_DEV void ppeg_wgrad_body(const float* __restrict__ x, const float* __restrict__ dy_, int S, int G, int D,
                            float* __restrict__ part, int bx, int by, int gx, int gy) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* win = lds;                  // [WIN][CS] x window
  float* dyt = lds + WIN * CS;       // [TR * TC][CS] dy tile
  const int nchunk = D / CW;
  const int tid = threadIdx.x, cq = tid & (NQ - 1), g = tid / NQ;   // g < 28: tap row g >> 2, tile rows 2 (g & 3) ..
  const int chunk = bx % nchunk, grp = bx / nchunk, b = by;
  const int ntc = (G + TC - 1) / TC, ngc = (ntc + WT - 1) / WT;
  const int tr = grp / ngc, tc0 = (grp % ngc) * WT;
  const float* xb = x + (size_t)b * S * D + D + chunk * CW;
  const float* gb = dy_ + (size_t)b * S * D + D + chunk * CW;
  const __amdgpu_buffer_rsrc_t rx = tm_rsrc(xb, (unsigned)(G * G * D) * 4u), rg = tm_rsrc(gb, (unsigned)(G * G * D) * 4u);
  const int tdy = g >> 2, rp = g & 3;   // g = 28..31: the bias sums of tile rows 2 (g - 28) ..
  const int r0 = tr * TR;
  f32x4 accw[KS];
#pragma unroll
  for (int dx = 0; dx < KS; ++dx) accw[dx] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int tc = tc0; tc < min(ntc, tc0 + WT); ++tc) {
    const int c0 = tc * TC;
    __syncthreads();   // the previous tile's LDS reads are done
    {
      const int q4 = cq * 4;
      const int cell = tid / NQ;   // 32 cells per pass, 2 passes
      f32x4 v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int cl = cell + 32 * u, rr = r0 + cl / TC, cc = c0 + cl % TC;
        v[u] = tm_bload4(rg, ((rr < G) & (cc < G)) ? (unsigned)((rr * G + cc) * D + q4) * 4u : TM_OOB);
      }
      load_window(win, rx, r0, c0, G, D, tid);
#pragma unroll
      for (int u = 0; u < 2; ++u) *(f32x4*)(dyt + (cell + 32 * u) * CS + q4) = v[u];
    }
    __syncthreads();
    if (g < 28) {
#pragma unroll 1
      for (int orow = 2 * rp; orow < 2 * rp + 2; ++orow) {
        f32x4 gv[TC], xv[WC];
#pragma unroll
        for (int j = 0; j < TC; ++j) gv[j] = ld4(dyt + (orow * TC + j) * CS + 4 * cq);
#pragma unroll
        for (int ic = 0; ic < WC; ++ic) xv[ic] = ld4(win + ((orow + tdy) * WC + ic) * CS + 4 * cq);
#pragma unroll
        for (int j = 0; j < TC; ++j)
#pragma unroll
          for (int dx = 0; dx < KS; ++dx)
#pragma unroll
            for (int e = 0; e < 4; ++e) accw[dx][e] = fmaf(gv[j][e], xv[j + dx][e], accw[dx][e]);
      }
    } else {
      const int bp = g - 28;
#pragma unroll
      for (int cell = 16 * bp; cell < 16 * bp + 16; ++cell) accw[0] += ld4(dyt + cell * CS + 4 * cq);
    }
  }
  // partial slab: the four tile-row pairs summed in a fixed order through LDS
  __syncthreads();
  float* red = lds;   // [4 row pairs][8 tap rows: 7 + bias][NQ][7][4]
  {
    const int pr = g < 28 ? rp : g - 28, trow = g < 28 ? tdy : 7;
    float* o = red + (((size_t)pr * 8 + trow) * NQ + cq) * 28;
#pragma unroll
    for (int dx = 0; dx < KS; ++dx) *(f32x4*)(o + dx * 4) = accw[dx];
  }
  __syncthreads();
  // four slab regions, each [Z][count] with Z = B * groups slabs (the deferred reduce sums a
  // region's slabs straight into one gradient): the folded 7x7 taps (= dw7), their 5x5 and 3x3
  // centres (the fold is a sum, so these are dw5 / dw3), and the bias sums (db7 = db5 = db3)
  const size_t Z = (size_t)gy * (gx / nchunk), z = (size_t)b * (gx / nchunk) + grp;
  float* p7 = part + z * D * NT;
  float* p5 = part + Z * D * NT + z * D * 25;
  float* p3 = part + Z * D * (NT + 25) + z * D * 9;
  float* pb = part + Z * D * (NT + 34) + z * D;
  for (int e = tid; e < CW * (NT + 1); e += 256) {
    const int cl = e / (NT + 1), tp = e - cl * (NT + 1);          // channel of the chunk, tap (49 = bias)
    const int q = cl >> 2, ce = cl & 3, ch = chunk * CW + cl;
    const int trow = tp == NT ? 7 : tp / KS, dx = tp == NT ? 0 : tp - (tp / KS) * KS;
    float s = 0.f;
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) s += red[(((size_t)pr * 8 + trow) * NQ + q) * 28 + dx * 4 + ce];
    if (tp == NT) {
      pb[ch] = s;
      continue;
    }
    p7[(size_t)ch * NT + tp] = s;
    if (trow >= 1 && trow <= 5 && dx >= 1 && dx <= 5) p5[(size_t)ch * 25 + (trow - 1) * 5 + dx - 1] = s;
    if (trow >= 2 && trow <= 4 && dx >= 2 && dx <= 4) p3[(size_t)ch * 9 + (trow - 2) * 3 + dx - 2] = s;
  }
}

// The backward's two independent parts as ONE launch (grid (nwg + nst, B), LDS of the larger):
// blocks [0, nwg) the weight gradient (three tiles each, so first), the rest the dx stencil.  One
// launch boundary fewer, and each part's tail runs under the other's blocks.
__global__ __launch_bounds__(256) void ppeg_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                      int S, int G, int D, const float* __restrict__ wf,
                                                      float* __restrict__ dx, DropPad dp, float* __restrict__ part,
                                                      int nwg) {
  if ((int)blockIdx.x < nwg) ppeg_wgrad_body(x, dy, S, G, D, part, blockIdx.x, blockIdx.y, nwg, gridDim.y);
  else ppeg_stencil_body<true>(dy, S, G, D, wf, nullptr, dx, dp, blockIdx.x - nwg, blockIdx.y);
}
constexpr int BWD_LDS = ST_LDS > WG_LDS ? ST_LDS : WG_LDS;

}  // namespace


extern "C" int tm_ppeg_fold(const float* w7, const float* b7, const float* w5, const float* b5, const float* w3,
                            const float* b3, int D, float* wfold, float* bfold, void* stream) {
  ppeg_fold_kernel<<<(D + 63) / 64, 64, 0, (hipStream_t)stream>>>(w7, b7, w5, b5, w3, b3, D, wfold, bfold);
  TM_CHECK_LAUNCH();
  return 0;
}

// x, y: [B, S, D] fp32 with S = 1 + G*G.  y must not alias x.
static int wgrad_groups(int G) {
  const int ntc = (G + TC - 1) / TC;
  return ((G + TR - 1) / TR) * ((ntc + WT - 1) / WT);
}

// x, y: [B, S, D] fp32 with S = 1 + G*G.  y must not alias x.
extern "C" int tm_ppeg_fwd(const float* x, int B, int G, int D, const float* wfold, const float* bfold, float* y,
                           void* stream) {
  TM_REQUIRE(x && y && x != y && D % CW == 0 && G > 0 && B > 0, "ppeg_fwd: bad args");
  // the tile kernels address one bag's grid through a buffer resource with 32-bit byte counts /
  // offsets: beyond 4 GiB per bag the hardware bounds check would turn loads into silent zeros
  TM_REQUIRE((1LL + (long long)G * G) * D * 4 < (1LL << 32), "ppeg_fwd: (1+G*G)*D*4 must be < 2^32 bytes per bag");
  const int ntiles = ((G + TR - 1) / TR) * ((G + TC - 1) / TC);
  ppeg_stencil_kernel<false><<<dim3(ntiles * (D / CW), B), 256, ST_LDS, (hipStream_t)stream>>>(
      x, 1 + G * G, G, D, wfold, bfold, y, DropPad{});
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_ppeg_bwd_workspace(int B, int G, int D) {
  return (long long)B * wgrad_groups(G) * D * (NT + 25 + 9 + 1) * (long long)sizeof(float);
}

// dy: [B,S,D] upstream gradient; x: PPEG input.  dx written (=); weight grads written.
extern "C" int tm_ppeg_bwd(const float* x, const float* dy, int B, int G, int D, const float* wfold, float* dx,
                           float* work, float* dw7, float* db7, float* dw5, float* db5, float* dw3, float* db3,
                           int dtype, void* dout, int n_pad, int pad, float p, uint64_t seed,
                           const uint64_t* seed_ptr, tm_reduce_queue* rq, void* stream) {
  TM_REQUIRE(x && dy && dx && dx != dy && D % CW == 0 && G > 0 && B > 0, "ppeg_bwd: bad args");
  TM_REQUIRE((1LL + (long long)G * G) * D * 4 < (1LL << 32), "ppeg_bwd: (1+G*G)*D*4 must be < 2^32 bytes per bag");
  TM_REQUIRE(!dout || ((dtype == TM_BF16 || dtype == TM_F32) && n_pad >= pad + 1 + G * G && pad >= 0),
             "ppeg_bwd: bad dropout-pad output");
  hipStream_t st = (hipStream_t)stream;
  const int S = 1 + G * G;
  const DropPad dp{dout, dtype, n_pad, pad, p, p > 0.f ? 1.f / (1.f - p) : 1.f, seed, seed_ptr};
  const int ntiles = ((G + TR - 1) / TR) * ((G + TC - 1) / TC);
  const int nwg = wgrad_groups(G) * (D / CW), nst = ntiles * (D / CW);
  ppeg_bwd_kernel<<<dim3(nwg + nst, B), 256, BWD_LDS, st>>>(x, dy, S, G, D, wfold, dx, dp, work, nwg);
  TM_CHECK_LAUNCH();
  // the weight-gradient slabs summed in slab order into the unfolded gradients (deferred into the
  // caller's queue when it has one: the flush that finalises the PPEG gradients is one launch)
  const int Z = B * wgrad_groups(G);
  const float* p5 = work + (size_t)Z * D * NT;
  const float* p3 = p5 + (size_t)Z * D * 25;
  const float* pb = p3 + (size_t)Z * D * 9;
  int rc = tm_splitk_reduce(work, dw7, Z, (long long)D * NT, 1.0f, 0, rq, stream);
  if (!rc) rc = tm_splitk_reduce(p5, dw5, Z, (long long)D * 25, 1.0f, 0, rq, stream);
  if (!rc) rc = tm_splitk_reduce(p3, dw3, Z, (long long)D * 9, 1.0f, 0, rq, stream);
  if (!rc) rc = tm_splitk_reduce(pb, db7, Z, D, 1.0f, 0, rq, stream);
  if (!rc) rc = tm_splitk_reduce(pb, db5, Z, D, 1.0f, 0, rq, stream);
  if (!rc) rc = tm_splitk_reduce(pb, db3, Z, D, 1.0f, 0, rq, stream);
  return rc;
}
