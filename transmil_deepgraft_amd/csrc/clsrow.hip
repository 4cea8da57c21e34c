// Class-row specialisation of the LAST TransLayer (code/models/TransMIL.py:195-204).
//
// TransMIL's output reads the last layer only through the class token: logits =
// _fc2(norm(h)[:, 0]) (:201-203).  So
//   forward:  of layer 2's attention output only the class row (sequence row `pad` of the
//             front-padded NystromAttention input, App. A eq. 1) is ever read: its A1 row
//             softmax(q_r k~^T) Y + conv33(v)_r, to_out (+ dropout) and the residual add;
//   backward: dL/dH3 is zero outside the class rows, so dropout, to_out and the A1 / conv33
//             backward of layer 2 see ONE non-zero query row per bag: dWo, dbo are outer
//             products, dq has one row, dk~ and dY are rank-1, dv has a 33-row window.
// Everything upstream of A1 (landmarks, A3, the pseudo-inverse, Y = Z W) and the whole
// dq~ / dk~ / dk / dv path through the pseudo-inverse and A3 stay dense, on the regular
// kernels.  The values computed here are the ones the dense kernels produce for these rows
// (the other rows' contributions are exact zeros), summed in a fixed order.
#include "common.h"
#include "head_bwd.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int NL = 256, DH = 64, TAPS = 33, HALF = 16;

TM_DEV float block_reduce_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
TM_DEV float block_reduce_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// thread j of a 256-thread block: s_j = q . k~_j (fp32 over T operands)
template <typename T>
TM_DEV float row_score(const T* __restrict__ qr, const T* __restrict__ klr) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < DH; c += 8) {
    const vec8<T> a = load8(qr + c), b = load8(klr + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) s = fmaf(to_f(a[e]), to_f(b[e]), s);
  }
  return s;
}

// out[d] (d = tid < 64, after the call) = sum_j w[j] M[j][d] for a [256][64] T matrix M and
// LDS weights w[256]: thread (g = tid >> 3, o = tid & 7) sums rows 8g..8g+7 of columns 8o..8o+7
// (eight 8-wide loads in flight), then 32 partials per column in index order.  block 256.
template <typename T>
TM_DEV float rows_dot(const float* w, const T* __restrict__ M, float (*part)[DH]) {
  const int tid = threadIdx.x, g = tid >> 3, o = (tid & 7) * 8;
  vec8<T> m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = load8(M + (size_t)(8 * g + i) * DH + o);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float wj = w[8 * g + i];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf(wj, to_f(m[i][e]), acc[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[g][o + e] = acc[e];
  __syncthreads();
  float s = 0.f;
  if (tid < DH)
    for (int gg = 0; gg < 32; ++gg) s += part[gg][tid];
  __syncthreads();
  return s;
}

// conv33 of one row: sum_tau w[tau] v[r + tau - 16][d] (d = tid < 64, after the call); thread
// (tg = tid >> 6, d) takes taps tg, tg + 4, ... (nine loads in flight).  block 256.
template <typename T>
TM_DEV float conv_row(const T* __restrict__ vb, const float* __restrict__ w, int r, int n, float (*part)[DH]) {
  const int tid = threadIdx.x, tg = tid >> 6, d = tid & 63;
  float x[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int tau = tg + 4 * i, t = r + tau - HALF;
    x[i] = (tau < TAPS && t >= 0 && t < n) ? to_f(vb[(size_t)t * DH + d]) : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 9; ++i)
    if (tg + 4 * i < TAPS) acc = fmaf(w[tg + 4 * i], x[i], acc);
  part[tg][d] = acc;
  __syncthreads();
  const float s = tid < DH ? (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]) : 0.f;
  __syncthreads();
  return s;
}

// Forward A1 row + conv33: grid (nbh), block 256.
//   p = softmax(q_r k~^T); merged[b][r][h*64 + d] = sum_j p_j Y[j][d] + sum_tau w[h][tau] v[r+tau-16][d]
template <typename T>
__global__ __launch_bounds__(256) void a1_row_fwd_kernel(const T* __restrict__ q, const T* __restrict__ v,
                                                         const T* __restrict__ kl_t, const T* __restrict__ y_t,
                                                         const float* __restrict__ wconv, int nh, int n, int r,
                                                         T* __restrict__ merged, float* __restrict__ lse1) {
  __shared__ float red[4];
  __shared__ float ps[NL];
  __shared__ float part[32][DH];
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh, tid = threadIdx.x;
  // the Y rows and the conv window are loaded up front, with the score operands (one memory round
  // trip instead of three: nothing below the first barrier issues a global load)
  const int g = tid >> 3, o = (tid & 7) * 8, tg = tid >> 6, d = tid & 63;
  vec8<T> ym[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ym[i] = load8(y_t + (size_t)bh * NL * DH + (size_t)(8 * g + i) * DH + o);
  float xc[9], wc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int tau = tg + 4 * i, t = r + tau - HALF;
    const bool in = tau < TAPS && t >= 0 && t < n;
    xc[i] = in ? to_f(v[((size_t)bh * n + t) * DH + d]) : 0.f;
    wc[i] = tau < TAPS ? wconv[h * TAPS + tau] : 0.f;
  }
  const T* qr = q + ((size_t)bh * n + r) * DH;
  const float s = row_score(qr, kl_t + ((size_t)bh * NL + tid) * DH);
  const float m = block_reduce_max(s, red);
  const float e = __expf(s - m);
  const float l = block_reduce_sum(e, red);
  ps[tid] = e / l;
  if (tid == 0) lse1[(size_t)bh * n + r] = m + __logf(l);
  __syncthreads();
  // sum_j p_j Y[j][d]: thread (g, o) its 8 rows x 8 columns, then the 32 row groups in order
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float wj = ps[8 * g + i];
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) acc[e2] = fmaf(wj, to_f(ym[i][e2]), acc[e2]);
  }
#pragma unroll
  for (int e2 = 0; e2 < 8; ++e2) part[g][o + e2] = acc[e2];
  __syncthreads();
  float py = 0.f;
  if (tid < DH)
    for (int gg = 0; gg < 32; ++gg) py += part[gg][tid];
  __syncthreads();
  // conv33: thread (tg, d) its taps tg, tg + 4, ..., then the 4 tap groups in order
  float ca = 0.f;
#pragma unroll
  for (int i = 0; i < 9; ++i)
    if (tg + 4 * i < TAPS) ca = fmaf(wc[i], xc[i], ca);
  part[tg][d] = ca;
  __syncthreads();
  const float cv = tid < DH ? (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]) : 0.f;
  if (tid < DH) merged[((size_t)b * n + r) * nh * DH + h * DH + tid] = from_f<T>(py + cv);
}

// to_out on the class rows: H3[b*S] = H2[b*S] + dropout(merged[b][r] Wo^T + bo) (row b*S of the
// dense epilogue's dropout hash).  grid (B, D / 4), block 256: one wave per output column, the
// lanes splitting the D-long dot 8 consecutive k at a time.
template <typename T>
__global__ __launch_bounds__(256) void cls_out_fwd_kernel(const T* __restrict__ merged, const T* __restrict__ wo,
                                                          const float* __restrict__ bo, const float* __restrict__ H2,
                                                          int n, int r, int S, int D, float p, float scale,
                                                          uint64_t seed0, const uint64_t* __restrict__ seed_ptr,
                                                          float* __restrict__ H3) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, c = blockIdx.y * 4 + (threadIdx.x >> 6);
  const T* mr = merged + ((size_t)b * n + r) * D;
  float s = 0.f;
  for (int k = lane * 8; k < D; k += 512) {
    const vec8<T> a = load8(mr + k), w = load8(wo + (size_t)c * D + k);
#pragma unroll
    for (int e = 0; e < 8; ++e) s = fmaf(to_f(a[e]), to_f(w[e]), s);
  }
  s = wave_sum(s);
  if (lane == 0) {
    float y = s + bo[c];
    const int row = b * S;
    if (p > 0.f) y = dropout_u01(effective_seed(seed0, seed_ptr), (uint32_t)row, (uint32_t)c) >= p ? y * scale : 0.f;
    H3[(size_t)row * D + c] = H2[(size_t)row * D + c] + y;
  }
}

// dout[b][c] = T(keep * scale * dH[b*S][c]) (as tm_dropout_bwd_pad), in fp32
template <typename T>
TM_DEV float dout_at(const float* __restrict__ dH, int b, int c, int S, int D, float p, float scale, uint64_t seed) {
  float v = dH[(size_t)b * S * D + c];
  if (p > 0.f) v = dropout_u01(seed, (uint32_t)(b * S), (uint32_t)c) >= p ? v * scale : 0.f;
  return to_f(from_f<T>(v));
}

// to_out backward on the class rows, three jobs by block range (bags summed in index order):
//   blocks [0, B*D/64):            dmerged[b][k] = T(sum_c dout[b][c] Wo[c][k])  (64 k per block)
//   blocks [B*D/64, +D/2):         dWo[c][k] = sum_b dout[b][c] merged[b][r][k]   (2 rows c per block)
//   the last block:                dbo[c] = sum_b dout[b][c]
// block 256.
// head + CrossEntropy backward folded into the class-row to_out backward (one bag, <= 4 classes,
// D = 512: the training step's fast path; layernorm.hip head_ce_bwd_kernel's B = 1 branch, same
// arithmetic): every block recomputes dL/dH3 at the class row (one wave, 8 channels per lane) from
// the saved softmax, x^ and rstd; the last block also writes it to dH and the head / norm gradients.
struct HeadBwd {
  const float* prob; const long long* label; const float* g;   // prob [C], label [1], dL/dloss [1]
  const float* xhat; const float* rstd; const float* gamma; const float* beta; const float* W;   // W [C][D]
  float* dW; float* dbias; float* dgamma; float* dbeta;
  int C;
};

template <typename T>
__global__ __launch_bounds__(256) void cls_out_bwd_kernel(const float* __restrict__ dH_in, const T* __restrict__ merged,
                                                          const T* __restrict__ wo, int B, int n, int r, int S, int D,
                                                          float p, float scale, uint64_t seed0,
                                                          const uint64_t* __restrict__ seed_ptr, float* __restrict__ dwo,
                                                          float* __restrict__ dbo, T* __restrict__ dmerged, HeadBwd hb) {
  extern __shared__ float dsh[];  // [D] dout of one bag, then [32][64] partials; head mode: [D] dL/dH3 after them
  const int tid = threadIdx.x, blk = blockIdx.x;
  const uint64_t seed = p > 0.f ? effective_seed(seed0, seed_ptr) : 0;
  const int nm = B * (D / 64);
  const float* dH = dH_in;
  if (hb.prob) {   // B = 1, D = 512 (host-checked): the class row's gradient from the head, in LDS
    float* hs = dsh + D + 32 * DH;
    if (tid < 64) {
      const bool last = blk == (int)gridDim.x - 1;
      head_bwd_b1<8>(hb.prob, hb.label, hb.g, nullptr, hb.C, hb.xhat, hb.rstd, hb.gamma, hb.beta, hb.W,
                     last ? hb.dW : nullptr, hb.dbias, hb.dgamma, hb.dbeta, last ? (float*)dH_in : nullptr, hs, tid);
    }
    __syncthreads();
    dH = hs;        // dout_at reads row b * S = 0 of it
  }
  if (blk < nm) {
    const int b = blk / (D / 64), k0 = (blk % (D / 64)) * 64;
    for (int c = tid; c < D; c += 256) dsh[c] = dout_at<T>(dH, b, c, S, D, p, scale, seed);
    __syncthreads();
    float(*part)[DH] = (float(*)[DH])(dsh + D);
    const int g = tid >> 3, o = k0 + (tid & 7) * 8, rows = D / 32;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c0 = g * rows; c0 < (g + 1) * rows; c0 += 8) {
      vec8<T> w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = load8(wo + (size_t)(c0 + i) * D + o);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(dsh[c0 + i], to_f(w[i][e]), acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[g][(tid & 7) * 8 + e] = acc[e];
    __syncthreads();
    if (tid < DH) {
      float s = 0.f;
      for (int gg = 0; gg < 32; ++gg) s += part[gg][tid];
      dmerged[(size_t)b * D + k0 + tid] = from_f<T>(s);
    }
    return;
  }
  if (blk < nm + D / 2) {
    const int c0 = (blk - nm) * 2;
    for (int i = tid; i < 2 * D; i += 256) {
      const int c = c0 + i / D, k = i % D;
      float s = 0.f;
      for (int b = 0; b < B; ++b) s = fmaf(dout_at<T>(dH, b, c, S, D, p, scale, seed), to_f(merged[((size_t)b * n + r) * D + k]), s);
      dwo[(size_t)c * D + k] = s;
    }
    return;
  }
  for (int c = tid; c < D; c += 256) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dout_at<T>(dH, b, c, S, D, p, scale, seed);
    dbo[c] = s;
  }
}

// A1 row + conv33 backward: grid (nbh, 4), block 256; every block recomputes p, dp and dS (cheap,
// L2-resident operands), then blockIdx.y picks one output: 0 dk~, 1 dY, 2 dq + dv window, 3 dwconv.  g = dmerged row (head slice), p = softmax
// row (lse1), dp_j = g . Y_j, D1 = p . dp, dS_j = p_j (dp_j - D1):
//   dq[bh][r] = sum_j dS_j k~_j  (the rest of dq is zero: the caller's buffer or dq_row consumers)
//   dkl[bh][j] = dS_j q_r (=)      dy[bh][j] = p_j g (=)
//   dv[bh][r + tau - 16] = w[h][tau] g   (the 33-row window)
//   dwconv[h][tau] = sum_b g_b . v_b[r + tau - 16]  (blocks of bag 0 sum the bags in order)
template <typename T>
__global__ __launch_bounds__(256) void a1_row_bwd_kernel(const T* __restrict__ dmerged, const T* __restrict__ q,
                                                         const T* __restrict__ v, const T* __restrict__ kl_t,
                                                         const T* __restrict__ y_t, const float* __restrict__ lse1,
                                                         const float* __restrict__ wconv, int B, int nh, int n, int r,
                                                         float* __restrict__ dq, float* __restrict__ dkl,
                                                         float* __restrict__ dy, T* __restrict__ dv,
                                                         float* __restrict__ dwconv) {
  __shared__ float red[4];
  __shared__ float gs[DH], qs[DH], dss[NL];
  __shared__ float part[32][DH];
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh, tid = threadIdx.x, D = nh * DH;
  const int lane = tid & 63, wave = tid >> 6;
  const T* qr = q + ((size_t)bh * n + r) * DH;
  if (tid < DH) {
    gs[tid] = to_f(dmerged[(size_t)b * D + h * DH + tid]);
    qs[tid] = to_f(qr[tid]);
  }
  __syncthreads();
  const float pj = __expf(row_score(qr, kl_t + ((size_t)bh * NL + tid) * DH) - lse1[(size_t)bh * n + r]);
  const T* yr = y_t + ((size_t)bh * NL + tid) * DH;
  float dp = 0.f;
#pragma unroll
  for (int c = 0; c < DH; c += 8) {
    const vec8<T> yv = load8(yr + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) dp = fmaf(gs[c + e], to_f(yv[e]), dp);
  }
  const float d1 = block_reduce_sum(pj * dp, red);
  const float ds = pj * (dp - d1);
  dss[tid] = ds;
  const int role = blockIdx.y;
  if (role == 0) {  // dk~ row j = dS_j q
    float* dklr = dkl + ((size_t)bh * NL + tid) * DH;
#pragma unroll
    for (int c = 0; c < DH; c += 4)
      *(f32x4*)(dklr + c) = (f32x4){ds * qs[c], ds * qs[c + 1], ds * qs[c + 2], ds * qs[c + 3]};
    return;
  }
  if (role == 1) {  // dY row j = p_j g
    float* dyr = dy + ((size_t)bh * NL + tid) * DH;
#pragma unroll
    for (int c = 0; c < DH; c += 4)
      *(f32x4*)(dyr + c) = (f32x4){pj * gs[c], pj * gs[c + 1], pj * gs[c + 2], pj * gs[c + 3]};
    return;
  }
  if (role == 2) {
    __syncthreads();
    const float dqv = rows_dot(dss, kl_t + (size_t)bh * NL * DH, part);
    if (tid < DH) dq[((size_t)bh * n + r) * DH + tid] = dqv;
    // conv33 backward window
    for (int i = tid; i < TAPS * DH; i += 256) {
      const int tau = i / DH, dd = i % DH, t = r + tau - HALF;
      if (t >= 0 && t < n) dv[((size_t)bh * n + t) * DH + dd] = from_f<T>(wconv[h * TAPS + tau] * gs[dd]);   // dv in T
    }
    return;
  }
  if (b == 0) {
    // wave w: taps w, w + 4, ...; lanes = d; bags in index order
    for (int tau = wave; tau < TAPS; tau += 4) {
      const int t = r + tau - HALF;
      float s = 0.f;
      if (t >= 0 && t < n)
        for (int bb = 0; bb < B; ++bb) {
          const float x = to_f(dmerged[(size_t)bb * D + h * DH + lane]) * to_f(v[(((size_t)bb * nh + h) * n + t) * DH + lane]);
          s += wave_sum(x);
        }
      if (lane == 0) dwconv[h * TAPS + tau] = s;
    }
  }
}

// The q operands of the class-row layer's q-part products (bf16 mode; see tm_cls_q_rows in the
// header).  Block (j, b), thread c = column (head c / 64, dim c % 64) of one operand row.
constexpr int QROWS = NL + 32;   // rows per bag: NL landmark rows, the class row, zero rows to a multiple of 32
// 512 threads, D = nh * 64 = 512 columns (host-checked).  Every load of the block is issued before
// the first add (16-B pieces): slab rows as 4 slab groups x 128 threads x 4 columns, segment rows as
// 8 row groups x 64 threads x 8 columns; the groups' partial sums are combined through LDS in a
// fixed order.
constexpr int QR_SLABS = 64;     // slabs per burst: 16 pieces per thread
__global__ __launch_bounds__(512) void cls_q_rows_kernel(const float* __restrict__ dql, const bf16* __restrict__ slab,
                                                         int nslabs, const float* __restrict__ dq,
                                                         const bf16* __restrict__ xn, int nh, int n, int r,
                                                         float* __restrict__ Aq, float* __restrict__ Xs) {
  constexpr int D = 512;
  __shared__ f32x4 sred[4][128];
  __shared__ float xred[8][D];
  const int j = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int l = n / NL;
  float* aout = Aq + ((size_t)b * QROWS + j) * D;
  float* xout = Xs + ((size_t)b * QROWS + j) * D;
  if (j > NL) {   // zero operand rows (block-uniform)
    aout[tid] = 0.f;
    xout[tid] = 0.f;
    return;
  }
  if (j == NL) {  // the class row
    const int hh = tid >> 6, d = tid & 63;
    aout[tid] = dq[(((size_t)b * nh + hh) * n + r) * DH + d];
    xout[tid] = (float)xn[((size_t)b * n + r) * D + tid];
    return;
  }
  // slab pieces: group g = tid / 128 takes slabs g, g + 4, ..; thread column c4 = 4 (tid % 128);
  // bursts of QR_SLABS slabs (one at the bench shape)
  const int g = tid >> 7, c4 = (tid & 127) * 4, hh = c4 >> 6, d = c4 & 63;
  const size_t ss = (size_t)gridDim.y * nh * NL * DH;
  const size_t o = (((size_t)b * nh + hh) * NL + j) * DH + d;
  // segment rows: group g8 = tid / 64 takes rows g8, g8 + 8, ..; thread columns 8 (tid % 64);
  // bursts of 64 rows (one at the bench shape, l = 33)
  const int g8 = tid >> 6, c8 = (tid & 63) * 8;
  const bf16* xr = xn + ((size_t)b * n + (size_t)j * l) * D + c8;
  constexpr int XR = 8;
  f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f};
  float x8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p0 = 0, t0 = 0; p0 < nslabs || t0 < l; p0 += QR_SLABS, t0 += 8 * XR) {
    f32x4 sp[QR_SLABS / 4];
#pragma unroll
    for (int i = 0; i < QR_SLABS / 4; ++i) {
      const int p = p0 + g + 4 * i;
      if (p < nslabs) {   // bf16 partials (tm_nys_a3_bwd_fused), summed in fp32
        const bf16x4 v = *(const bf16x4*)(slab + p * ss + o);
        sp[i] = (f32x4){(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
      } else {
        sp[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
    bf16x8 xp[XR];
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int t = t0 + g8 + 8 * i;
      xp[i] = t < l ? *(const bf16x8*)(xr + (size_t)t * D) : (bf16x8){};
    }
#pragma unroll
    for (int i = 0; i < QR_SLABS / 4; ++i) s += sp[i];
#pragma unroll
    for (int i = 0; i < XR; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) x8[e] += (float)xp[i][e];
  }
  sred[g][tid & 127] = s;
#pragma unroll
  for (int e = 0; e < 8; ++e) xred[g8][c8 + e] = x8[e];
  __syncthreads();
  if (tid < 128) {
    const f32x4 q = *(const f32x4*)(dql + o) + ((sred[0][tid] + sred[1][tid]) + (sred[2][tid] + sred[3][tid]));
    *(f32x4*)(aout + c4) = q / (float)l;
  }
  float xs = xred[0][tid];
#pragma unroll
  for (int i = 1; i < 8; ++i) xs += xred[i][tid];
  xout[tid] = xs;
}

}  // namespace

#define TM_CLS_DISPATCH(dt, CALL)                                 \
  if ((dt) == TM_BF16) { using T = bf16; CALL; }                  \
  else if ((dt) == TM_F32) { using T = float; CALL; }             \
  else { tm_set_error("clsrow: dtype must be TM_F32 or TM_BF16"); return 1; }

extern "C" int tm_cls_a1_row_fwd(int dtype, const void* q, const void* v, const void* kl_t, const void* y_t,
                                 const float* wconv, int nbh, int nh, int n, int r, void* merged, float* lse1,
                                 void* stream) {
  TM_REQUIRE(q && v && kl_t && y_t && wconv && merged && lse1 && nbh > 0 && nh > 0 && nbh % nh == 0,
             "cls_a1_row_fwd: bad args");
  TM_REQUIRE(n % NL == 0 && r >= 0 && r < n, "cls_a1_row_fwd: bad row / n");
  TM_CLS_DISPATCH(dtype, (a1_row_fwd_kernel<T><<<nbh, 256, 0, (hipStream_t)stream>>>(
                             (const T*)q, (const T*)v, (const T*)kl_t, (const T*)y_t, wconv, nh, n, r, (T*)merged, lse1)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_cls_out_fwd(int dtype, const void* merged, const void* wo, const float* bo, const float* H2, int B,
                              int n, int r, int S, int D, float p, uint64_t seed,
                              const uint64_t* seed_ptr, float* H3, void* stream) {
  TM_REQUIRE(merged && wo && bo && H2 && H3 && B > 0 && D % 64 == 0, "cls_out_fwd: bad args");
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  TM_CLS_DISPATCH(dtype, (cls_out_fwd_kernel<T><<<dim3(B, D / 4), 256, 0, (hipStream_t)stream>>>(
                             (const T*)merged, (const T*)wo, bo, H2, n, r, S, D, p, scale, seed, seed_ptr, H3)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_cls_out_bwd(int dtype, const float* dH, const void* merged, const void* wo, int B, int n, int r,
                              int S, int D, float p, uint64_t seed, const uint64_t* seed_ptr,
                              float* dwo, float* dbo, void* dmerged, void* stream) {
  TM_REQUIRE(dH && merged && wo && dwo && dbo && dmerged && B > 0 && D % 64 == 0, "cls_out_bwd: bad args");
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  TM_REQUIRE(D <= 8192, "cls_out_bwd: D <= 8192");
  const int blocks = B * (D / 64) + D / 2 + 1;
  const size_t sm = (size_t)(D + 32 * 64) * sizeof(float);
  TM_CLS_DISPATCH(dtype, (cls_out_bwd_kernel<T><<<blocks, 256, sm, (hipStream_t)stream>>>(
                             dH, (const T*)merged, (const T*)wo, B, n, r, S, D, p, scale, seed, seed_ptr, dwo, dbo, (T*)dmerged,
                             HeadBwd{})));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_cls_head_out_bwd(int dtype, const float* prob, const long long* label, const float* gloss, int C,
                                   const float* xhat, const float* rstd, const float* gamma, const float* beta,
                                   const float* W, float* dW, float* dbias, float* dgamma, float* dbeta, float* dH,
                                   const void* merged, const void* wo, int n, int r, int S, int D, float p,
                                   uint64_t seed, const uint64_t* seed_ptr, float* dwo, float* dbo, void* dmerged,
                                   void* stream) {
  TM_REQUIRE(prob && label && gloss && xhat && rstd && gamma && beta && W && dW && dbias && dgamma && dbeta,
             "cls_head_out_bwd: bad head args");
  TM_REQUIRE(dH && merged && wo && dwo && dbo && dmerged, "cls_head_out_bwd: bad args");
  TM_REQUIRE(D == 512 && C >= 1 && C <= 4, "cls_head_out_bwd: one bag, D = 512, <= 4 classes");
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int blocks = (D / 64) + D / 2 + 1;
  const size_t sm = (size_t)(2 * D + 32 * 64) * sizeof(float);
  const HeadBwd hb{prob, label, gloss, xhat, rstd, gamma, beta, W, dW, dbias, dgamma, dbeta, C};
  TM_CLS_DISPATCH(dtype, (cls_out_bwd_kernel<T><<<blocks, 256, sm, (hipStream_t)stream>>>(
                             dH, (const T*)merged, (const T*)wo, 1, n, r, S, D, p, scale, seed, seed_ptr, dwo, dbo, (T*)dmerged,
                             hb)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_cls_a1_row_bwd(int dtype, const void* dmerged, const void* q, const void* v, const void* kl_t,
                                 const void* y_t, const float* lse1, const float* wconv, int B, int nh, int n, int r,
                                 float* dq, float* dkl, float* dy, void* dv, float* dwconv, void* stream) {
  TM_REQUIRE(dmerged && q && v && kl_t && y_t && lse1 && wconv && dq && dkl && dy && dv && dwconv && B > 0 && nh > 0,
             "cls_a1_row_bwd: bad args");
  TM_REQUIRE(n % NL == 0 && r >= 0 && r < n, "cls_a1_row_bwd: bad row / n");
  TM_CLS_DISPATCH(dtype, (a1_row_bwd_kernel<T><<<dim3(B * nh, 4), 256, 0, (hipStream_t)stream>>>(
                             (const T*)dmerged, (const T*)q, (const T*)v, (const T*)kl_t, (const T*)y_t, lse1, wconv,
                             B, nh, n, r, dq, dkl, dy, (T*)dv, dwconv)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_cls_q_rows(const float* dql, const void* slab, int nslabs, const float* dq, const void* xn, int B,
                             int nh, int n, int r, float* Aq, float* Xs, void* stream) {
  TM_REQUIRE(dql && dq && xn && Aq && Xs && B > 0 && nh * DH == 512 && (nslabs == 0 || slab),
             "cls_q_rows: bad args (nh * 64 must be 512)");
  TM_REQUIRE(n % NL == 0 && r >= 0 && r < n && nslabs >= 0, "cls_q_rows: bad row / n / slab count");
  cls_q_rows_kernel<<<dim3(QROWS, B), 512, 0, (hipStream_t)stream>>>(dql, (const bf16*)slab, nslabs, dq, (const bf16*)xn, nh, n, r,
                                                                     Aq, Xs);
  TM_CHECK_LAUNCH();
  return 0;
}
