// NystromAttention core (SURVEY.md section 8 App. A eq. 4-9), forward and backward.
//
// Replaces the arithmetic of the third-party `nystrom_attention.NystromAttention`
// called at code/models/TransMIL.py:26-34,47 (not vendored).
// Fixed geometry: dim_head = 64, num_landmarks = 256 (TransLayer always builds
// dim_head = dim/8, num_landmarks = dim/2 with dim = 512, code/models/TransMIL.py:26-31).
//
// Layouts in HBM (bh = bag*heads + head, n = n' = padded length, l = n/256):
//   q, k, v        [3][B*h][n][64]  T   (q pre-scaled by dim_head^-0.5)
//   ql, kl         [B*h][256][64]   fp32 (+ T copies for the MFMA paths)
//   merged out     [B][n][h*64]     T   (input of to_out)
//
// Forward (reassociated):  out = softmax(q kl^T) . (Z . (softmax(ql k^T) . v)) + conv33(v)
// i.e. attn1 @ (Z @ (attn3 @ v)) instead of (attn1 @ Z) @ (attn3 @ v): saves
// n*256*256*2 flop per head (8.86 GF/layer at N=8192); results agree to fp32
// rounding (tests/test_parity_gpu.py).
//
// Kernels
//   landmarks        segment means of q, k (eq. 4)                 HBM-bound
//   sim2_softmax     A2 = softmax(ql kl^T) (eq. 5-6), fp32          tiny
//   a3_fwd/combine   W = softmax(ql k^T) v, split over key blocks   flash-decode style
//   a1_fwd           softmax(q kl^T) Y + conv(v) -> merged rows     one pass, 256 keys
//   conv_bwd         conv33 backward + D1 = rowsum(dO * O_att)
//   attn_bwd<MODE>   shared flash-style backward for the A1 and A3 products
//   assemble_dqkv    dq, dk, dv + landmark terms -> [B][n][3*h*64]
#include <algorithm>
#include <type_traits>
#include "common.h"
#include "a3_combine.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int DH = 64;     // dim_head
constexpr int NL = 256;    // landmarks
constexpr int TAPS = 33;   // residual conv kernel
constexpr int HALF = 16;   // conv padding

// LDS row strides (elements).  Keys [256][KROW]: 144 B (bf16) / 272 B (f32) rows
// -> conflict-free ds_read_b128 for 16 consecutive rows.
// Values, bf16: natural [256 keys][VROW = 80] (160-B rows: the transposing
// ds_read_b64_tr_b16 of 4 keys x 16 d hits 64 distinct banks per 32-lane half);
// fp32 (parity mode, no 32-bit transposing read): values^T [64][VROW = 260].
template <typename T> struct Lay {
  static constexpr int KROW = DH + 16 / (int)sizeof(T);    // 72 bf16 / 68 f32
  static constexpr int VROW = sizeof(T) == 2 ? 80 : NL + 4;
  static constexpr int VELEMS = sizeof(T) == 2 ? NL * VROW : DH * VROW;
};

template <typename T> union Chunk16 { f32x4 raw; T e[16 / sizeof(T)]; };

TM_DEV long long hoff(long long bh, int nh, long long bag_stride, long long head_stride) {
  return (bh / nh) * bag_stride + (bh % nh) * head_stride;
}

// ---------------------------------------------------------------------------
// landmarks: out[bh][j][d] = sum_{t<l} x[bh][j*l+t][d] / l ; grid (nbh, 32), block 256: thread
// (landmark 8 blockIdx.y + tid / 32, d octet (tid / 4) % 8, row quarter tid % 4) sums its quarter of
// the l rows with 8-wide loads (all of them in flight for l <= 36), then the 4 quarters meet by
// xor shuffles in a fixed order.
template <typename T>
__global__ __launch_bounds__(256) void landmarks_kernel(const T* __restrict__ q, const T* __restrict__ k, int n,
                                                        int l, float* __restrict__ ql, float* __restrict__ kl,
                                                        T* __restrict__ ql_t, T* __restrict__ kl_t) {
  const int bh = blockIdx.x, tid = threadIdx.x, tq = tid & 3, o = ((tid >> 2) & 7) * 8;
  const int j = blockIdx.y * 8 + (tid >> 5);
  const int per = (l + 3) / 4, t0 = tq * per, t1 = min(l, t0 + per);
  const T* qp = q + ((size_t)bh * n + (size_t)j * l) * DH + o;
  const T* kp = k + ((size_t)bh * n + (size_t)j * l) * DH + o;
  float sq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, sk[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int t = t0; t < t1; t += 9) {
    vec8<T> a[9], b[9];
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int tt = min(t + u, t1 - 1);
      a[u] = load8(qp + (size_t)tt * DH);
      b[u] = load8(kp + (size_t)tt * DH);
    }
#pragma unroll
    for (int u = 0; u < 9; ++u)
      if (t + u < t1)
#pragma unroll
        for (int e = 0; e < 8; ++e) { sq[e] += to_f(a[u][e]); sk[e] += to_f(b[u][e]); }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sq[e] += __shfl_xor(sq[e], 1, 64); sk[e] += __shfl_xor(sk[e], 1, 64);
    sq[e] += __shfl_xor(sq[e], 2, 64); sk[e] += __shfl_xor(sk[e], 2, 64);
  }
  if (tq) return;
  const float inv_l = (float)l;
  const size_t oo = ((size_t)bh * NL + j) * DH + o;
  float vq[8], vk[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { vq[e] = sq[e] / inv_l; vk[e] = sk[e] / inv_l; }
  *(f32x4*)(ql + oo) = (f32x4){vq[0], vq[1], vq[2], vq[3]};
  *(f32x4*)(ql + oo + 4) = (f32x4){vq[4], vq[5], vq[6], vq[7]};
  *(f32x4*)(kl + oo) = (f32x4){vk[0], vk[1], vk[2], vk[3]};
  *(f32x4*)(kl + oo + 4) = (f32x4){vk[4], vk[5], vk[6], vk[7]};
  vec8<T> tq8, tk8;
#pragma unroll
  for (int e = 0; e < 8; ++e) { tq8[e] = from_f<T>(vq[e]); tk8[e] = from_f<T>(vk[e]); }
  store8<T>(ql_t + oo, tq8);
  store8<T>(kl_t + oo, tk8);
}

// ---------------------------------------------------------------------------
// A2 = softmax_j(ql_i . kl_j), fp32 FMA.  grid (nbh, 256 / S2_ROWS), block 256: S2_ROWS rows per
// block, thread = column j.  k~ of the head arrives by coalesced 16-B loads (every load in flight
// at once) and is transposed into LDS ([64][260] fp32: thread j reads column j, conflict-free);
// the q~ rows are LDS broadcasts.
// a2s (optional): the same values as bf16 hi / lo planes (hi = bf16(a), lo = bf16(a - hi); lo plane at
// a2s + nbh * 256 * 256), the operand format of the split pseudo-inverse chain (pinv_split.hip).
constexpr int S2_ROWS = 8;

// A2 rows by ONE wave each (shared by sim2_softmax_kernel and the fused A3 forward, so both write
// the same bits): the wave computes RW rows -- q~ rows qrow0, qrow0 + qstep, .. of `qs` ([rows][64]
// fp32 in LDS) against the head's k~ in LDS as a row image [256][64] fp32 whose row j keeps its 16-B
// chunk c at slot c ^ (j & 15) (kimg: filled by LDS-DMA, k2_stage_dma) -- lane l owning columns l,
// l + 64, l + 128, l + 192 and reading each 4-d chunk of a row as one conflict-free 16-B read.  The
// logits keep the sequential fmaf order over d; the row max and sum are in-wave reductions (no LDS
// partials, no barrier: the 256-thread-per-row form spent ~9.7k of the A3 forward's cycles in its
// three barriers and cross-wave exchanges).  Output row k at o0 + k ostep.
constexpr int S2_KIMG = NL * DH;   // floats of the k~ row image

// k~ of head bh (kl [nbh][256][64] fp32) into the swizzled row image kimg by LDS-DMA: 64 pieces of
// 1 KB (4 rows), `nwaves` waves; lane L of a piece writes row 4 piece + L / 16, slot L % 16, i.e.
// fetches the row's chunk (L % 16) ^ (row & 15).  Completion: the issuing waves' vmcnt + a barrier.
TM_DEV void k2_stage_dma(float* kimg, const float* __restrict__ kl, int bh, int wave, int nwaves, int lane) {
  typedef __attribute__((address_space(3))) void lds_t;
  typedef __attribute__((address_space(1))) void glb_t;
  const float* kb = kl + (size_t)bh * NL * DH;
  for (int piece = wave; piece < 64; piece += nwaves) {
    const int row = piece * 4 + (lane >> 4), slot = lane & 15;
    __builtin_amdgcn_global_load_lds((glb_t*)(kb + (size_t)row * DH + (slot ^ (row & 15)) * 4),
                                     (lds_t*)(kimg + piece * 256), 16, 0, 0);
  }
}

template <int RW>
TM_DEV void sim2_wave_rows(const float* kimg, const float* qs, int qrow0, int qstep, int lane, float* __restrict__ a2,
                           bf16* __restrict__ a2s, size_t o0, size_t ostep, size_t plane) {
  float s[RW][4];
#pragma unroll
  for (int k = 0; k < RW; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) s[k][i] = 0.f;
  const int sw = lane & 15;   // (lane + 64 i) & 15
#pragma unroll 4
  for (int c = 0; c < DH; c += 4) {
    float kv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 t = *(const f32x4*)(kimg + (lane + 64 * i) * DH + (((c >> 2) ^ sw) << 2));
#pragma unroll
      for (int e = 0; e < 4; ++e) kv[i][e] = t[e];
    }
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const f32x4 q4 = *(const f32x4*)(qs + (qrow0 + k * qstep) * DH + c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[k][i] = fmaf(q4[e], kv[i][e], s[k][i]);
    }
  }
#pragma unroll
  for (int k = 0; k < RW; ++k) {
    const float m = wave_max_dpp(fmaxf(fmaxf(s[k][0], s[k][1]), fmaxf(s[k][2], s[k][3])));
#pragma unroll
    for (int i = 0; i < 4; ++i) s[k][i] = __expf(s[k][i] - m);
    const float tot = wave_sum_dpp((s[k][0] + s[k][1]) + (s[k][2] + s[k][3]));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t o = o0 + (size_t)k * ostep + lane + 64 * i;
      const float v = s[k][i] / tot;
      a2[o] = v;
      if (a2s) {
        const bf16 hi = (bf16)v;
        a2s[o] = hi;
        a2s[o + plane] = (bf16)(v - (float)hi);
      }
    }
  }
}

__global__ __launch_bounds__(256) void sim2_softmax_kernel(const float* __restrict__ ql, const float* __restrict__ kl,
                                                           float* __restrict__ a2, bf16* __restrict__ a2s) {
  const int bh = blockIdx.x, i0 = blockIdx.y * S2_ROWS, j = threadIdx.x;
  // one LDS array (the k~ row image, then the q~ rows): a second __shared__ object beside an LDS-DMA
  // target can make hipcc drain the DMA early (cdna_hip_programming.md section 5, trap 4(a))
  __shared__ __attribute__((aligned(16))) float lds[S2_KIMG + S2_ROWS * DH];
  float* kimg = lds;
  float* qs = lds + S2_KIMG;
  const int w = j >> 6;
  k2_stage_dma(kimg, kl, bh, w, 4, j & 63);
  {
    static_assert(S2_ROWS * DH % 256 == 0, "sim2: q~ rows per thread");
    constexpr int QE = S2_ROWS * DH / 256;
    float qv[QE];
#pragma unroll
    for (int u = 0; u < QE; ++u) qv[u] = ql[((size_t)bh * NL + i0) * DH + u * 256 + j];
#pragma unroll
    for (int u = 0; u < QE; ++u) qs[u * 256 + j] = qv[u];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's k~ pieces landed
  __syncthreads();
  // wave w: rows i0 + w and i0 + w + 4
  sim2_wave_rows<S2_ROWS / 4>(kimg, qs, w, 4, j & 63, a2, a2s, ((size_t)bh * NL + i0 + w) * NL, (size_t)4 * NL,
                              (size_t)gridDim.x * NL * NL);
}

// bench-mode A2 = softmax_j(ql_i . kl_j) on the MFMA: the logits as bf16x3 products (x = hi + lo,
// hi*hi + hi*lo + lo*hi, fp32 accumulation: ~2^-17 relative, the precision of the split planes
// the chain then reads).  grid (nbh, 8), block 512: rows 32 by .. of one head; wave w owns
// columns 32 w .. 32 w + 31 (one 32x32 tile, 4 k-steps x 3 MFMAs).  Every operand load is issued
// before the first MFMA (64 floats per lane); row max / sum: 32-lane shuffles, then the 8 waves'
// partials through LDS in a fixed order.  Writes A2 (fp32) and its hi / lo planes.
#ifdef TM_DIAG
__global__ __launch_bounds__(512) void sim2_softmax_mfma_kernel(const float* __restrict__ ql,
                                                                const float* __restrict__ kl, float* __restrict__ a2,
                                                                bf16* __restrict__ a2s) {
  __shared__ float red[2][8][32];
  const int bh = blockIdx.x, r0 = blockIdx.y * 32, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5, c0 = wave * 32;
  const float* qa = ql + ((size_t)bh * NL + r0 + r) * DH + 8 * h;
  const float* kb = kl + ((size_t)bh * NL + c0 + r) * DH + 8 * h;
  f32x4 av[8], bv[8];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    av[2 * s] = *(const f32x4*)(qa + 16 * s);
    av[2 * s + 1] = *(const f32x4*)(qa + 16 * s + 4);
    bv[2 * s] = *(const f32x4*)(kb + 16 * s);
    bv[2 * s + 1] = *(const f32x4*)(kb + 16 * s + 4);
  }
  f32x16 acc = (f32x16){};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 ah, al, bhi, blo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = e < 4 ? av[2 * s][e] : av[2 * s + 1][e - 4];
      const float y = e < 4 ? bv[2 * s][e] : bv[2 * s + 1][e - 4];
      ah[e] = (bf16)x;
      al[e] = (bf16)(x - (float)ah[e]);
      bhi[e] = (bf16)y;
      blo[e] = (bf16)(y - (float)bhi[e]);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bhi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, blo, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bhi, acc, 0, 0, 0);
  }
  // row i (reg i, half h) holds columns c0 + (lane & 31): max / sum over the 32 lanes of the half
  auto half_max = [](float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
  };
  auto half_sum = [](float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float m = half_max(acc[i]);
    if (r == 0) red[0][wave][acc_row(i, h)] = m;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = acc_row(i, h);
    float m = red[0][0][row];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = fmaxf(m, red[0][w][row]);
    acc[i] = __expf(acc[i] - m);
    const float t = half_sum(acc[i]);
    if (r == 0) red[1][wave][row] = t;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = acc_row(i, h);
    const float tot = ((red[1][0][row] + red[1][1][row]) + (red[1][2][row] + red[1][3][row])) +
                      ((red[1][4][row] + red[1][5][row]) + (red[1][6][row] + red[1][7][row]));
    const size_t o = ((size_t)bh * NL + r0 + row) * NL + c0 + r;
    const float v = acc[i] / tot;
    a2[o] = v;
    const bf16 hi = (bf16)v;
    a2s[o] = hi;
    a2s[o + (size_t)gridDim.x * NL * NL] = (bf16)(v - (float)hi);
  }
}

#endif  // TM_DIAG

// dS2 = A2 * (dA2 - rowsum(dA2 * A2)); grid (nbh*256/4), block 256 (one wave per row)
__global__ void softmax_bwd_rows_kernel(const float* __restrict__ a, const float* __restrict__ da,
                                        float* __restrict__ ds, int rows) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const f32x4 av = *(const f32x4*)(a + (size_t)r * NL + lane * 4);
  const f32x4 dv = *(const f32x4*)(da + (size_t)r * NL + lane * 4);
  const float s = wave_sum(av[0] * dv[0] + av[1] * dv[1] + av[2] * dv[2] + av[3] * dv[3]);
  f32x4 o;
  o[0] = av[0] * (dv[0] - s); o[1] = av[1] * (dv[1] - s); o[2] = av[2] * (dv[2] - s); o[3] = av[3] * (dv[3] - s);
  *(f32x4*)(ds + (size_t)r * NL + lane * 4) = o;
}

// A operand of O^T = V^T P^T for d tile dt and the 16-key step starting at key kb:
// element j of lane (r, h) = V[kb + 8(j>>2) + 4h + (j&3)][dt*32 + r]  (acc_k_index order).
template <typename T> TM_DEV vec8<T> value_frag(const T* vs, int dt, int kb, int lane);
template <> TM_DEV bf16x8 value_frag<bf16>(const bf16* vs, int dt, int kb, int lane) {
  // natural [key][80] layout, two transposing reads of 4 keys x 16 d
  constexpr int VROW = Lay<bf16>::VROW;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int d = dt * 32 + (g & 1) * 16 + 4 * p;
  const int key = kb + 4 * (g >> 1) + q;
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(vs + key * VROW + d));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(vs + (key + 8) * VROW + d));
  return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
template <> TM_DEV f32x8 value_frag<float>(const float* vt, int dt, int kb, int lane) {
  // transposed [d][260] layout
  constexpr int VROW = Lay<float>::VROW;
  const float* row = vt + (dt * 32 + (lane & 31)) * VROW + kb + 4 * (lane >> 5);
  const f32x4 lo = *(const f32x4*)row, hi = *(const f32x4*)(row + 8);
  return (f32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}


// ---------------------------------------------------------------------------
// Shared forward block: one wave, 32 queries (B-operand fragments qf), 256 keys in
// LDS (ks[key][KROW]), values^T in LDS (vt[d][VROW]).  Returns unnormalised O^T
// (2 tiles: d 0-31, 32-63; col = query) plus per-query max and sum.
constexpr float LOG2E = 1.4426950408889634f;

// 16-element max as v_max3_f32 triples (8 instructions instead of 15)
TM_DEV float max3f(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }
TM_DEV float tree_max16(const f32x16& x) {
  const float m0 = max3f(x[0], x[1], x[2]), m1 = max3f(x[3], x[4], x[5]), m2 = max3f(x[6], x[7], x[8]);
  const float m3 = max3f(x[9], x[10], x[11]), m4 = max3f(x[12], x[13], x[14]);
  return __builtin_fmaxf(max3f(m0, m1, m2), max3f(m3, m4, x[15]));
}
// 16-element sum with packed adds (v_pk_add_f32: two lanes of the tree per instruction)
TM_DEV float tree_sum16(const f32x16& x) {
  f32x2 a[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    a[i] = (f32x2){x[2 * i], x[2 * i + 1]} + (f32x2){x[2 * i + 8], x[2 * i + 9]};
  a[0] += a[2];
  a[1] += a[3];
  a[0] += a[1];
  return a[0][0] + a[0][1];
}

template <typename T>
TM_DEV void attn_fwd_wave(const T* ks, const T* vt, const vec8<T> (&qf)[4], f32x16 (&o)[2], float& mx, float& sum,
                          int lane) {
  constexpr int KROW = Lay<T>::KROW;
  const int r = lane & 31, h = lane >> 5;
  f32x16 s[8];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    s[kt] = (f32x16){};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const vec8<T> a = load8(ks + (kt * 32 + r) * KROW + st * 16 + 8 * h);
      mma16(s[kt], a, qf[st]);
    }
  }
  // row max and sum as balanced trees (a 128-long dependent fmaxf / add chain per lane
  // costs its full latency), exp as exp2 of one fma: p = 2^(s log2e - m log2e)
  float mk[8];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) mk[kt] = tree_max16(s[kt]);
  float m = fmaxf(fmaxf(fmaxf(mk[0], mk[1]), fmaxf(mk[2], mk[3])), fmaxf(fmaxf(mk[4], mk[5]), fmaxf(mk[6], mk[7])));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float ml = m * LOG2E;
  float lk[8];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[kt][i] = __builtin_amdgcn_exp2f(fmaf(s[kt][i], LOG2E, -ml));
    lk[kt] = tree_sum16(s[kt]);
  }
  float l = ((lk[0] + lk[1]) + (lk[2] + lk[3])) + ((lk[4] + lk[5]) + (lk[6] + lk[7]));
  l += __shfl_xor(l, 32, 64);
  mx = m;
  sum = l;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    o[dt] = (f32x16){};
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
        mma16(o[dt], value_frag<T>(vt, dt, kt * 32 + 16 * sp, lane), acc_as_operand<T>(s[kt], sp));
  }
}

// A [256][64] T tile (row stride 64) held in registers between its global loads and its
// LDS writes: a compile-time count of 16-B pieces per thread, so every load of the tile is
// issued before the first wait (a runtime-bounded `for (i = tid; ...)` loop let the compiler
// pipeline only the first few and serialise the rest, one HBM/L2 round trip each).
template <typename T, int NT = 256>
struct TileRegs {
  static constexpr int E = 16 / sizeof(T), PER_ROW = DH / E, PER = NL * PER_ROW / NT;
  f32x4 r[PER];
  TM_DEV void load(const T* src, int tid) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + NT * j;
      r[j] = *(const f32x4*)(src + (size_t)(i / PER_ROW) * DH + (i % PER_ROW) * E);
    }
  }
  // keys: ks[key][KROW]
  TM_DEV void store_keys(T* ks, int tid) const {
    constexpr int KROW = Lay<T>::KROW;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + NT * j;
      *(f32x4*)(ks + (i / PER_ROW) * KROW + (i % PER_ROW) * E) = r[j];
    }
  }
  // values in the layout of Lay<T> (bf16 natural [key][VROW], fp32 transposed [d][VROW])
  TM_DEV void store_values(T* vs, int tid) const {
    constexpr int VROW = Lay<T>::VROW;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + NT * j, key = i / PER_ROW, d0 = (i % PER_ROW) * E;
      if constexpr (sizeof(T) == 2) {
        *(f32x4*)(vs + key * VROW + d0) = r[j];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) vs[(d0 + e) * VROW + key] = r[j][e];
      }
    }
  }
};

// stage T rows [256][64] (row stride 64) into ks[key][KROW]
template <typename T>
TM_DEV void stage_keys_t(T* ks, const T* src, int tid) {
  TileRegs<T> t;
  t.load(src, tid);
  t.store_keys(ks, tid);
}
// stage values [256 keys][64] (T rows, stride 64) into the value layout of Lay<T>
template <typename T>
TM_DEV void stage_values(T* vs, const T* src, int tid) {
  TileRegs<T> t;
  t.load(src, tid);
  t.store_values(vs, tid);
}

// ---------------------------------------------------------------------------
// A1 path forward.  grid (n/128, nbh), block 256 (4 waves x 32 queries).
//   merged[bag][t][head*64+d] = softmax_j(q_t . kl_j) . Y_j  + sum_tau w[head][tau] v[t+tau-16][d]
//   lse1[bh][t] saved for backward.
constexpr int A1_VS = 66;  // conv window row stride (floats): a wave's 2 query groups hit distinct banks
constexpr int A1_WIN_ITEMS = (128 + 2 * HALF) * 8 / 256;
constexpr size_t A1_EPI_BYTES = (128 * 68 + (128 + 2 * HALF) * A1_VS) * sizeof(float);

template <typename T, int VAR = 0>   // VAR (ablation): 1 = no conv taps, 2 = no MFMA phase
__global__ __launch_bounds__(256, 2) void a1_fwd_kernel(const T* __restrict__ q, const T* __restrict__ v,
                                                     const T* __restrict__ kl_t, const T* __restrict__ y_t,
                                                     const float* __restrict__ wconv, int n, int nh,
                                                     T* __restrict__ merged, float* __restrict__ lse1) {
  constexpr int KROW = Lay<T>::KROW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* ks = (T*)smem;                                  // [256][KROW]
  T* vt = ks + NL * KROW;                            // values (Lay<T>)
  float* ost = (float*)smem;                         // reuse: [128][68] fp32 after the MFMA phase
  const int bh = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int head = bh % nh, bag = bh / nh;
  const int t0 = blockIdx.x * 128;
  const T* qb = q + (size_t)bh * n * DH;
  const T* vb = v + (size_t)bh * n * DH;
  vec8<T> qf[4];
  const int qrow = t0 + wave * 32 + r;
  // conv window: v rows [t0 - 16, t0 + 144) of this head (5 x 16 B per thread)
  vec8<T> vwin[A1_WIN_ITEMS];
  auto load_window = [&]() {
#pragma unroll
    for (int i = 0; i < A1_WIN_ITEMS; ++i) {
      const int it = tid + 256 * i, row = it >> 3, src = t0 - HALF + row;
      if (src >= 0 && src < n) vwin[i] = load8(vb + (size_t)src * DH + (it & 7) * 8);
      else vwin[i] = vec8<T>{};
    }
  };
  if constexpr (sizeof(T) == 2) {
    // one burst: landmark keys, Y and this wave's query fragments (the conv window is
    // requested after the MFMA phase: held across it, it would cost the second wave per SIMD)
    TileRegs<T> kr, yr;
    kr.load(kl_t + (size_t)bh * NL * DH, tid);
    yr.load(y_t + (size_t)bh * NL * DH, tid);
#pragma unroll
    for (int st = 0; st < 4; ++st) qf[st] = load8(qb + (size_t)qrow * DH + st * 16 + 8 * h);
    kr.store_keys(ks, tid);
    yr.store_values(vt, tid);
  } else {
    stage_keys_t<T>(ks, kl_t + (size_t)bh * NL * DH, tid);
    stage_values<T>(vt, y_t + (size_t)bh * NL * DH, tid);
#pragma unroll
    for (int st = 0; st < 4; ++st) qf[st] = load8(qb + (size_t)qrow * DH + st * 16 + 8 * h);
  }
  __syncthreads();
  f32x16 o[2];
  float mx, sum;
  if constexpr (VAR == 2) {
    o[0] = (f32x16){}; o[1] = (f32x16){};
    mx = to_f(qf[0][0]); sum = 1.f + to_f(ks[lane]) + to_f(vt[lane]);
  } else {
    attn_fwd_wave<T>(ks, vt, qf, o, mx, sum, lane);
  }
  if (h == 0) lse1[(size_t)bh * n + qrow] = mx + __logf(sum);
  const float inv = 1.0f / sum;
  // the conv window is requested now, overlapping the normalisation / LDS round trip below
  load_window();
  __syncthreads();  // everyone done reading ks/vt
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = dt * 32 + 8 * g4 + 4 * h;
      f32x4 val;
      val[0] = o[dt][4 * g4] * inv; val[1] = o[dt][4 * g4 + 1] * inv;
      val[2] = o[dt][4 * g4 + 2] * inv; val[3] = o[dt][4 * g4 + 3] * inv;
      *(f32x4*)(ost + (wave * 32 + r) * 68 + d0) = val;
    }
  float* vs = ost + 128 * 68;  // [160][A1_VS] fp32 window
#pragma unroll
  for (int i = 0; i < A1_WIN_ITEMS; ++i) {
    const int it = tid + 256 * i, row = it >> 3, dc = (it & 7) * 8;
#pragma unroll
    for (int e = 0; e < 8; e += 2)
      *(float2*)(vs + row * A1_VS + dc + e) = make_float2(to_f(vwin[i][e]), to_f(vwin[i][e + 1]));
  }
  __syncthreads();
  // conv residual, register-blocked: thread = (16 consecutive queries, 2 d); every window
  // row is read once from LDS and feeds up to 16 outputs.
  if constexpr (VAR != 1) {
    const int dp = tid & 31, qb = tid >> 5;
    const float* wc = wconv + head * TAPS;
    float w[TAPS];
#pragma unroll
    for (int tau = 0; tau < TAPS; ++tau) w[tau] = wc[tau];
    float2 acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = *(const float2*)(ost + (qb * 16 + j) * 68 + 2 * dp);
#pragma unroll
    for (int i = 0; i < 16 + 2 * HALF; ++i) {
      const float2 x = *(const float2*)(vs + (qb * 16 + i) * A1_VS + 2 * dp);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int tau = i - j;
        if (tau >= 0 && tau < TAPS) {
          acc[j].x = fmaf(w[tau], x.x, acc[j].x);
          acc[j].y = fmaf(w[tau], x.y, acc[j].y);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) *(float2*)(ost + (qb * 16 + j) * 68 + 2 * dp) = acc[j];
    __syncthreads();
  }
  // coalesced store: item = (query, 8 d)
  for (int it = tid; it < 128 * 8; it += 256) {
    const int ql = it >> 3, dc = (it & 7) * 8, t = t0 + ql;
    vec8<T> outv;
#pragma unroll
    for (int e = 0; e < 8; ++e) outv[e] = from_f<T>(ost[ql * 68 + dc + e]);
    store8(merged + ((size_t)bag * n + t) * (nh * DH) + head * DH + dc, outv);
  }
}

// ---------------------------------------------------------------------------
// A1 path forward, bf16 (bench mode): one workgroup of 8 waves per CU; the landmark keys
// and Y are staged ONCE per workgroup and each wave walks 32-query chunks of its head.
// grid = (W, nbh) with W = min(256 / nbh, n / 32) workgroups per head and the head's n / 32
// chunks split evenly over them, so at N = 8192 every CU holds one workgroup (the
// 128-query-per-workgroup form launched 528 blocks on 512 slots: a second round for 16).
// The 33-tap residual conv runs on the MFMA: per chunk (queries t0..t0+31)
//   O^T[d][q] += sum_j V[t0 - 16 + j][d] * band[j][q],  band[j][q] = w[j - q] (0 <= j - q < 33)
// over the workgroup's v window: rows [32 c_begin - 16, 32 c_end + 16) copied HBM -> LDS by
// LDS-DMA (global_load_lds, no VGPRs) in the prologue and left in flight through the first
// attention phase (v is read 1.1-1.2x, not the 2x of per-chunk windows).  Rows outside
// [0, n) are fetched clamped and masked in the band instead.  The band fragments of
// interior chunks are one shared LDS table; the first / last chunk of a head build theirs.
// LDS: keys [256][72] + Y [256][80] + window [<=320][64] + 4 output stages [32][72] + band
// table + taps = 140 KB.  One wave per SIMD (512 registers): the wave overlaps its own MFMA
// and VALU work instead of two waves running the same phases in lockstep.
constexpr int A1P_WAVES = 4;                                            // one wave per SIMD: 512 registers
constexpr int A1P_MAXCH = 9;                                            // chunks per workgroup (host-checked)
constexpr int A1P_WROWS = A1P_MAXCH * 32 + 32;                          // 320 window rows
constexpr int A1P_OROW = DH + 8;                                        // output stage row (bf16): 144 B
constexpr size_t A1P_KS = (size_t)NL * Lay<bf16>::KROW * 2;             // 36864
constexpr size_t A1P_VT = (size_t)NL * Lay<bf16>::VROW * 2;             // 40960
constexpr size_t A1P_WIN = (size_t)A1P_WROWS * DH * 2;                  // 40960
constexpr size_t A1P_OST = (size_t)32 * A1P_OROW * 2;                   // 4608 per wave
constexpr size_t A1P_WIN_OFF = A1P_KS + A1P_VT;
constexpr size_t A1P_OST_OFF = A1P_WIN_OFF + A1P_WIN;
constexpr size_t A1P_BAND_OFF = A1P_OST_OFF + A1P_WAVES * A1P_OST;      // [4][64] x 16 B
constexpr size_t A1P_TAPS_OFF = A1P_BAND_OFF + 4 * 64 * 16;
constexpr size_t A1P_BYTES = A1P_TAPS_OFF + 128 * sizeof(float);        // 162304

// diagnostic stamps (VAR 9 build only): [block][wave][slot] s_memtime, read by tm_debug_a1_stamps
__device__ unsigned long long g_a1_stamps[512 * 8 * 8];
template <int VAR>
TM_DEV void a1p_stamp(int slot, int wave) {
  if constexpr (VAR == 9) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if ((threadIdx.x & 63) == 0)
      g_a1_stamps[((blockIdx.y * gridDim.x + blockIdx.x) * 8 + wave) * 8 + slot] = t;
  }
}

TM_DEV void wave_lds_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// A operand of the conv product: window rows kb.. (acc_k_index order, as value_frag)
TM_DEV bf16x8 a1p_window_frag(const bf16* win, int dt, int kb, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int d = dt * 32 + (g & 1) * 16 + 4 * p;
  const int key = kb + 4 * (g >> 1) + q;
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(win + key * DH + d));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(win + (key + 8) * DH + d));
  return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// attn_fwd_wave with the per-tile work interleaved for the scheduler: the max tree of score
// tile kt beside the MFMAs of tile kt + 1, the exp / sum / bf16 packing of tile kt beside its
// P.V MFMAs (the two-phase form ran the MFMA and VALU phases back to back).
TM_DEV void attn_fwd_wave_il(const bf16* ks, const bf16* vt, const bf16x8 (&qf)[4], f32x16 (&o)[2], float& mx,
                             float& sum, int lane) {
  constexpr int KROW = Lay<bf16>::KROW;
  const int r = lane & 31, h = lane >> 5;
  f32x16 s[8];
  float mk[8];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    s[kt] = (f32x16){};
#pragma unroll
    for (int st = 0; st < 4; ++st) mma16(s[kt], load8(ks + (kt * 32 + r) * KROW + st * 16 + 8 * h), qf[st]);
    mk[kt] = tree_max16(s[kt]);
  }
  float m = fmaxf(fmaxf(fmaxf(mk[0], mk[1]), fmaxf(mk[2], mk[3])), fmaxf(fmaxf(mk[4], mk[5]), fmaxf(mk[6], mk[7])));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float ml = m * LOG2E;
  o[0] = (f32x16){};
  o[1] = (f32x16){};
  float lk[8];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[kt][i] = __builtin_amdgcn_exp2f(fmaf(s[kt][i], LOG2E, -ml));
    lk[kt] = tree_sum16(s[kt]);
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      const bf16x8 p = acc_as_operand<bf16>(s[kt], sp);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) mma16(o[dt], value_frag<bf16>(vt, dt, kt * 32 + 16 * sp, lane), p);
    }
  }
  float l = ((lk[0] + lk[1]) + (lk[2] + lk[3])) + ((lk[4] + lk[5]) + (lk[6] + lk[7]));
  l += __shfl_xor(l, 32, 64);
  mx = m;
  sum = l;
}

// attn_fwd_wave_il with its LDS fragments software-pipelined one tile ahead (one wave per SIMD
// has no partner wave to hide a read's latency: the il form waited on every key / value read
// right before its MFMA).  Key fragments of tile kt + 1 and value fragments of tile kt + 1 are
// issued before the MFMAs of tile kt; the max tree of tile kt - 1 and the exp / pack of tile
// kt + 1 run beside them.  Same arithmetic, same order of every sum: bitwise the il results
// (scripts/dev/fwd_pipe_ab.py: 14.4 -> 13.8 us per call at the bench shape).
TM_DEV void attn_fwd_wave_pipe(const bf16* ks, const bf16* vt, const bf16x8 (&qf)[4], f32x16 (&o)[2], float& mx,
                               float& sum, int lane) {
  constexpr int KROW = Lay<bf16>::KROW;
  const int r = lane & 31, h = lane >> 5;
  f32x16 s[8];
  float mk[8];
  bf16x8 kf[2][4];
#pragma unroll
  for (int st = 0; st < 4; ++st) kf[0][st] = load8(ks + r * KROW + st * 16 + 8 * h);
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    if (kt < 7) {
#pragma unroll
      for (int st = 0; st < 4; ++st) kf[(kt + 1) & 1][st] = load8(ks + ((kt + 1) * 32 + r) * KROW + st * 16 + 8 * h);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead (the scheduler sinks reads to their use)
    s[kt] = (f32x16){};
#pragma unroll
    for (int st = 0; st < 4; ++st) mma16(s[kt], kf[kt & 1][st], qf[st]);
    if (kt > 0) mk[kt - 1] = tree_max16(s[kt - 1]);
    __builtin_amdgcn_sched_barrier(0);
  }
  mk[7] = tree_max16(s[7]);
  float m = fmaxf(fmaxf(fmaxf(mk[0], mk[1]), fmaxf(mk[2], mk[3])), fmaxf(fmaxf(mk[4], mk[5]), fmaxf(mk[6], mk[7])));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float ml = m * LOG2E;
  o[0] = (f32x16){};
  o[1] = (f32x16){};
  float lk[8];
  bf16x8 vf[2][4], pf[2][2];
#pragma unroll
  for (int sp = 0; sp < 2; ++sp)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) vf[0][2 * sp + dt] = value_frag<bf16>(vt, dt, 16 * sp, lane);
#pragma unroll
  for (int i = 0; i < 16; ++i) s[0][i] = __builtin_amdgcn_exp2f(fmaf(s[0][i], LOG2E, -ml));
  lk[0] = tree_sum16(s[0]);
  pf[0][0] = acc_as_operand<bf16>(s[0], 0);
  pf[0][1] = acc_as_operand<bf16>(s[0], 1);
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    const int b = kt & 1, nb = b ^ 1;
    if (kt < 7) {
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) vf[nb][2 * sp + dt] = value_frag<bf16>(vt, dt, (kt + 1) * 32 + 16 * sp, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) mma16(o[dt], vf[b][2 * sp + dt], pf[b][sp]);
    if (kt < 7) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[kt + 1][i] = __builtin_amdgcn_exp2f(fmaf(s[kt + 1][i], LOG2E, -ml));
      lk[kt + 1] = tree_sum16(s[kt + 1]);
      pf[nb][0] = acc_as_operand<bf16>(s[kt + 1], 0);
      pf[nb][1] = acc_as_operand<bf16>(s[kt + 1], 1);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  float l = ((lk[0] + lk[1]) + (lk[2] + lk[3])) + ((lk[4] + lk[5]) + (lk[6] + lk[7]));
  l += __shfl_xor(l, 32, 64);
  mx = m;
  sum = l;
}

template <int VAR = 0>  // ablation: 1 no conv MFMAs, 2 no attention phase, 3 prologue only, 9 stamps,
                        // 6 the earlier attention form (attn_fwd_wave_il: reads just in time)
__global__ __launch_bounds__(256) void a1_fwd_bf16_kernel(const bf16* __restrict__ q, const bf16* __restrict__ v,
                                                          const bf16* __restrict__ kl_t, const bf16* __restrict__ y_t,
                                                          const float* __restrict__ wconv, int n, int nh, int wpg,
                                                          bf16* __restrict__ merged, float* __restrict__ lse1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* ks = (bf16*)smem;
  bf16* vt = (bf16*)(smem + A1P_KS);
  bf16* win = (bf16*)(smem + A1P_WIN_OFF);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  bf16* ost = (bf16*)(smem + A1P_OST_OFF + wave * A1P_OST);
  bf16x8* band_tab = (bf16x8*)(smem + A1P_BAND_OFF);
  float* taps = (float*)(smem + A1P_TAPS_OFF);
  const int bh = blockIdx.y, gi = blockIdx.x;
  const int head = bh % nh, bag = bh / nh;
  const int cph = n / 32;                          // 32-query chunks of this head
  const int c_begin = (int)((long long)gi * cph / wpg), c_end = (int)((long long)(gi + 1) * cph / wpg);
  const int w0 = c_begin * 32 - HALF;              // sequence row of window row 0
  const int wrows = (c_end - c_begin) * 32 + 2 * HALF;
  const bf16* qb = q + (size_t)bh * n * DH;
  const bf16* vb = v + (size_t)bh * n * DH;
  const int ld = nh * DH;
  a1p_stamp<VAR>(0, wave);

  // ---- prologue: keys, Y, taps and this wave's first query fragments through registers;
  //      the v window by LDS-DMA, left in flight through the first attention phase ----
  int c = c_begin + wave;
  bf16x8 qf[4];
  if (c < c_end) {
#pragma unroll
    for (int st = 0; st < 4; ++st) qf[st] = load8(qb + (size_t)(c * 32 + r) * DH + st * 16 + 8 * h);
  }
  TileRegs<bf16, 256> kr, yr;
  kr.load(kl_t + (size_t)bh * NL * DH, tid);
  yr.load(y_t + (size_t)bh * NL * DH, tid);
  float tapv = 0.f;
  if (tid < 128) {
    const int tau = tid - 32;  // taps[k] = w[k - 32], zero outside the filter
    if (tau >= 0 && tau < TAPS) tapv = wconv[head * TAPS + tau];
  }
  {
    typedef __attribute__((address_space(3))) void lds_t;
    typedef __attribute__((address_space(1))) void glb_t;
#pragma unroll
    for (int i = 0; i < A1P_WROWS * 8 / 256; ++i) {
      const int pc = i * 256 + tid, row = pc >> 3;  // 16-B piece pc of the window image
      if (i * 32 < wrows) {                         // wave-uniform: 8 rows per wave-instruction
        const int src = min(max(w0 + row, 0), n - 1);
        __builtin_amdgcn_global_load_lds((glb_t*)(vb + (size_t)src * DH + (pc & 7) * 8),
                                         (lds_t*)(win + (size_t)(i * 256 + wave * 64) * 8), 16, 0, 0);
      }
    }
  }
  kr.store_keys(ks, tid);
  yr.store_values(vt, tid);
  if (tid < 128) taps[tid] = tapv;
  __syncthreads();  // taps visible
  {  // interior band fragments: element jj of lane (rr, hh), k-step s = wave
    const int s = tid >> 6, ln = tid & 63, rr = ln & 31, hh = ln >> 5;
    bf16x8 b;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) b[jj] = (bf16)taps[16 * s + 8 * (jj >> 2) + 4 * hh + (jj & 3) - rr + 32];
    band_tab[s * 64 + ln] = b;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // keys / Y / band table in LDS; the window DMA may still be in flight
  a1p_stamp<VAR>(1, wave);
  if constexpr (VAR == 3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (c < c_end && lane == 0) lse1[(size_t)bh * n + c * 32] = to_f(ks[tid]) + to_f(vt[tid]) + to_f(qf[0][0]);
    return;
  }

  bool first = true;
  for (;;) {
    const bool active = c < c_end;
    const int t0 = c * 32;
    f32x16 o[2];
    float mx = 0.f, sum = 1.f;
    if (active) {
      if constexpr (VAR == 2) {
        o[0] = (f32x16){}; o[1] = (f32x16){};
        mx = to_f(qf[0][0]);
      } else {
        if constexpr (VAR == 6) attn_fwd_wave_il(ks, vt, qf, o, mx, sum, lane);
        else attn_fwd_wave_pipe(ks, vt, qf, o, mx, sum, lane);
      }
    }
    if (first) a1p_stamp<VAR>(2, wave);
    const int cn = c + A1P_WAVES;
    if (cn < c_end) {
#pragma unroll
      for (int st = 0; st < 4; ++st) qf[st] = load8(qb + (size_t)(cn * 32 + r) * DH + st * 16 + 8 * h);
    }
    if (first) {
      // every wave's window pieces have landed (the next chunk's 4 query loads may not)
      if (cn < c_end) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      first = false;
      a1p_stamp<VAR>(3, wave);
    }
    if (!active) break;
    // band fragments from the shared table.  At the sequence ends the window rows outside
    // [0, n) are exactly one k-step: rows j < 16 (k-step 0) for t0 = 0, rows j >= 48 (k-step 3)
    // for the last chunk -- those fragments are zeroed.
    bf16x8 band[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) band[s] = band_tab[s * 64 + lane];
    if (t0 == 0) band[0] = bf16x8{};
    if (t0 + 32 == n) band[3] = bf16x8{};
    const float inv = 1.0f / sum;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[dt][i] *= inv;
    if constexpr (VAR != 1) {
      const bf16* wc = win + (size_t)(t0 - HALF - w0) * DH;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int s = 0; s < 4; ++s) mma16(o[dt], a1p_window_frag(wc, dt, 16 * s, lane), band[s]);
    }
    if (c == c_begin + wave) a1p_stamp<VAR>(4, wave);
    if (h == 0) lse1[(size_t)bh * n + t0 + r] = mx + __logf(sum);
    // O^T registers -> [32 q][72] bf16 wave stage -> full 128-B row stores, 16 B per lane
    // (row-per-lane 8-B stores are store-issue bound)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        bf16x4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = (bf16)o[dt][4 * g4 + e];
        *(bf16x4*)(ost + r * A1P_OROW + dt * 32 + 8 * g4 + 4 * h) = pk;
      }
    wave_lds_fence();
    f32x4 ov[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = lane + 64 * i;
      ov[i] = *(const f32x4*)(ost + (p >> 3) * A1P_OROW + (p & 7) * 8);
    }
    bf16* dst = merged + ((size_t)bag * n + t0) * ld + head * DH;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = lane + 64 * i;
      *(f32x4*)(dst + (size_t)(p >> 3) * ld + (p & 7) * 8) = ov[i];
    }
    wave_lds_fence();  // stage read back before the next chunk rewrites it
    if (c == c_begin + wave) a1p_stamp<VAR>(5, wave);
    c = cn;
    if (c >= c_end) break;
  }
  a1p_stamp<VAR>(6, wave);
}

// ---------------------------------------------------------------------------
// A3 path forward, one 256-key block x 128 landmark queries per workgroup.
// grid (n/256, nbh, 2), block 256.
//   part_o[kb][bh][q][d] = sum_{keys in kb} exp(s - m_kb) v ; part_ml[kb][bh][q] = (m, l)
template <typename T>
__global__ __launch_bounds__(256, 2) void a3_fwd_kernel(const float* __restrict__ ql, const T* __restrict__ k,
                                                     const T* __restrict__ v, int n, float* __restrict__ part_o,
                                                     float* __restrict__ part_m, float* __restrict__ part_l) {
  constexpr int KROW = Lay<T>::KROW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* ks = (T*)smem;
  T* vt = ks + NL * KROW;
  const int kb = blockIdx.x, bh = blockIdx.y, nbh = gridDim.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const size_t kv_off = ((size_t)bh * n + (size_t)kb * NL) * DH;
  const int qi = blockIdx.z * 128 + wave * 32 + r;  // query half per workgroup
  vec8<T> qf[4];
  if constexpr (sizeof(T) == 2) {
    TileRegs<T> kr, vr;  // one burst: keys, values, query fragments
    kr.load(k + kv_off, tid);
    vr.load(v + kv_off, tid);
#pragma unroll
    for (int st = 0; st < 4; ++st) qf[st] = cvt8<T>(ql + ((size_t)bh * NL + qi) * DH + st * 16 + 8 * h);
    kr.store_keys(ks, tid);
    vr.store_values(vt, tid);
  } else {
    stage_keys_t<T>(ks, k + kv_off, tid);
    stage_values<T>(vt, v + kv_off, tid);
#pragma unroll
    for (int st = 0; st < 4; ++st) qf[st] = cvt8<T>(ql + ((size_t)bh * NL + qi) * DH + st * 16 + 8 * h);
  }
  __syncthreads();
  {
    f32x16 o[2];
    float mx, sum;
    attn_fwd_wave<T>(ks, vt, qf, o, mx, sum, lane);
    const size_t pidx = ((size_t)kb * nbh + bh) * NL + qi;
    if (h == 0) { part_m[pidx] = mx; part_l[pidx] = sum; }
    float* po = part_o + pidx * DH;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        f32x4 val;
        val[0] = o[dt][4 * g4]; val[1] = o[dt][4 * g4 + 1]; val[2] = o[dt][4 * g4 + 2]; val[3] = o[dt][4 * g4 + 3];
        *(f32x4*)(po + dt * 32 + 8 * g4 + 4 * h) = val;
      }
  }
}

// A3 path forward, bf16 (bench mode): one 512-thread workgroup per CU holds ALL 256 landmark
// queries of its head (8 waves x 32) against an even share of the head's keys, so k and v are read
// from HBM once (the 128-query form read them twice) and a head has P (<= 32) partials instead of
// 2 x n/256 half-slabs.  grid (P, nbh); workgroup p takes the 32-key sub-blocks
// [p S32 / P, (p + 1) S32 / P) (S32 = n / 32) in chunks of up to A3V_G sub-blocks, double-buffered
// in LDS (k [key][72], v [key][80]): the next chunk's 16-B pieces are requested into registers before
// the current chunk's scores, so its HBM round trip overlaps them; online softmax across chunks.
//   part_o[p][bh][q][d] = sum_keys exp(s - m) v ; part_m, part_l[p][bh][q] = (m, l)
constexpr int A3V_G = 5;                                           // sub-blocks (32 keys) per chunk
constexpr int A3V_KEYS = A3V_G * 32;
constexpr size_t A3V_KS = (size_t)A3V_KEYS * Lay<bf16>::KROW * 2;  // 23040 B
constexpr size_t A3V_BUF = A3V_KS + (size_t)A3V_KEYS * Lay<bf16>::VROW * 2;   // + 25600 B
constexpr size_t A3V_BYTES = 2 * A3V_BUF;                          // two chunk buffers: 97280 B
constexpr int A3V_PIECES = (A3V_KEYS * 8 + 511) / 512;             // 16-B pieces per thread per operand

// partials per head of the v2 kernel
inline int a3v_splits(int nbh, int n) { return std::max(1, std::min(n / 32, tm_cu_count() / std::max(nbh, 1))); }

// S2R > 0: the workgroup also writes A2 = softmax(q~ k~^T) rows p * 2 S2R .. + 2 S2R - 1 of its head
// (sim2_wave_rows, rows dealt over the 8 waves; host-checked 2 S2R P == 256) before its first key
// chunk is staged: the k~ / q~ loads go out ahead of the chunk's, so the rows are computed while the
// chunk is in flight, and the separate sim2 launch disappears from the step.
struct Sim2Out { const float* kl; float* a2; bf16* a2s; };
template <int ST = 0, int S2R = 0>   // ST: diagnostic s_memtime stamps (g_a1_stamps)
__global__ __launch_bounds__(512) void a3_fwd_v2_kernel(const float* __restrict__ ql, const bf16* __restrict__ k,
                                                        const bf16* __restrict__ v, int n, int P,
                                                        bf16* __restrict__ part_o, float* __restrict__ part_m,
                                                        float* __restrict__ part_l, Sim2Out s2) {
  constexpr int KROW = Lay<bf16>::KROW, VROW = Lay<bf16>::VROW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.x, bh = blockIdx.y, nbh = gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  auto stamp = [&](int slot) { if (ST) a1p_stamp<ST ? 9 : 0>(slot, wave); };
  stamp(0);
  const int S32 = n / 32;
  const int sb0 = (int)((long long)p * S32 / P), sb1 = (int)((long long)(p + 1) * S32 / P);
  const int qi = wave * 32 + r;
  const bf16* kh = k + (size_t)bh * n * DH;
  const bf16* vh = v + (size_t)bh * n * DH;
  f32x4 kr[A3V_PIECES], vr[A3V_PIECES];
  // the 16-B pieces of the chunk starting at sub-block c0 (rows clamped into the chunk)
  auto fetch = [&](int c0) {
    const int rows = min(A3V_G, sb1 - c0) * 32;
#pragma unroll
    for (int j = 0; j < A3V_PIECES; ++j) {
      const int i = tid + 512 * j, row = min(i >> 3, rows - 1), c = (i & 7) * 8;
      const size_t o = ((size_t)c0 * 32 + row) * DH + c;
      kr[j] = *(const f32x4*)(kh + o);
      vr[j] = *(const f32x4*)(vh + o);
    }
  };
  auto stage = [&](int c0, int buf) {
    const int rows = min(A3V_G, sb1 - c0) * 32;
    bf16* ks = (bf16*)(smem + buf * A3V_BUF);
    bf16* vs = (bf16*)(smem + buf * A3V_BUF + A3V_KS);
#pragma unroll
    for (int j = 0; j < A3V_PIECES; ++j) {
      const int i = tid + 512 * j, row = i >> 3, c = (i & 7) * 8;
      if (row < rows) {
        *(f32x4*)(ks + row * KROW + c) = kr[j];
        *(f32x4*)(vs + row * VROW + c) = vr[j];
      }
    }
  };
  // fused A2 rows (S2R > 0): computed AFTER the key loop, from k~ loaded into registers during the
  // first key chunk (so its L2 round trip hides under the chunk's MFMAs) and written into the LDS the
  // chunk buffers leave free; the A2 rows then cost only the tail's LDS staging and arithmetic (the
  // prologue form made the first key chunk wait for them: +5 us per call)
  constexpr int S2Q = S2R > 0 ? S2R * DH / 256 : 1;
  float q2[S2Q];
  f32x4 k2[S2R > 0 ? 8 : 1];
  const int g2 = tid >> 8, j2 = tid & 255, r2 = p * 2 * S2R + g2 * S2R;
  fetch(sb0);
  if constexpr (S2R > 0) {
#pragma unroll
    for (int u = 0; u < S2Q; ++u) q2[u] = ql[((size_t)bh * NL + r2) * DH + u * 256 + j2];
  }
  bf16x8 qf[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) qf[st] = cvt8<bf16>(ql + ((size_t)bh * NL + qi) * DH + st * 16 + 8 * h);
  stamp(1);
  stage(sb0, 0);
  __syncthreads();
  stamp(2);
  float m_run = -INFINITY, l_run = 0.f;
  f32x16 o[2];
  o[0] = (f32x16){};
  o[1] = (f32x16){};
  int buf = 0;
  for (int c0 = sb0; c0 < sb1; c0 += A3V_G) {
    const int ng = min(A3V_G, sb1 - c0);
    const bool more = c0 + A3V_G < sb1;
    if (more) fetch(c0 + A3V_G);   // in flight through this chunk's scores
    if constexpr (S2R > 0) {
      if (c0 == sb0) {   // k~ of the head for the A2 rows of the tail (16-B pieces: row p / 16, d 4 (p % 16))
        const float* kb = s2.kl + (size_t)bh * NL * DH;
#pragma unroll
        for (int u = 0; u < 8; ++u) k2[u] = *(const f32x4*)(kb + (size_t)(u * 512 + tid) * 4);
      }
    }
    const bf16* ks = (const bf16*)(smem + buf * A3V_BUF);
    const bf16* vs = (const bf16*)(smem + buf * A3V_BUF + A3V_KS);
    f32x16 s[A3V_G];   // S^T tiles (rows = keys, col = this lane's query)
#pragma unroll
    for (int kt = 0; kt < A3V_G; ++kt) {
      s[kt] = (f32x16){};
      if (kt < ng) {
#pragma unroll
        for (int st = 0; st < 4; ++st) mma16(s[kt], load8(ks + (kt * 32 + r) * KROW + st * 16 + 8 * h), qf[st]);
      }
    }
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < A3V_G; ++kt)
      if (kt < ng) m = fmaxf(m, tree_max16(s[kt]));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float m_new = fmaxf(m_run, m);
    const float corr = __builtin_amdgcn_exp2f((m_run - m_new) * LOG2E);   // 0 on the first chunk
    const float ml = m_new * LOG2E;
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < A3V_G; ++kt) {
      if (kt < ng) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kt][i] = __builtin_amdgcn_exp2f(fmaf(s[kt][i], LOG2E, -ml));
        l += tree_sum16(s[kt]);
      }
    }
    l += __shfl_xor(l, 32, 64);
    l_run = l_run * corr + l;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      o[dt] *= corr;
#pragma unroll
      for (int kt = 0; kt < A3V_G; ++kt)
        if (kt < ng) {
#pragma unroll
          for (int sp = 0; sp < 2; ++sp)
            mma16(o[dt], value_frag<bf16>(vs, dt, kt * 32 + 16 * sp, lane), acc_as_operand<bf16>(s[kt], sp));
        }
    }
    if (c0 == sb0) stamp(3);
    if (more) {
      stage(c0 + A3V_G, buf ^ 1);   // the other buffer: last read two chunks ago, before the barrier below
      __syncthreads();
      buf ^= 1;
    }
    if (c0 == sb0) stamp(4);
  }
  stamp(5);
  if constexpr (S2R > 0) {
    // (before the partial stores: a barrier behind them would wait for their write-back)
    __syncthreads();   // every wave is done with the chunk buffers
    float* kimg = (float*)smem;                        // k~ row image [256][64]: row j's chunk c at slot c ^ (j & 15)
    float* qs = kimg + S2_KIMG + g2 * S2R * DH;        // [2 S2R rows][64]: group g2's rows at g2 S2R
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int pc = u * 512 + tid, row = pc >> 4, c = pc & 15;
      *(f32x4*)(kimg + row * DH + ((c ^ (row & 15)) << 2)) = k2[u];
    }
#pragma unroll
    for (int u = 0; u < S2Q; ++u) qs[u * 256 + j2] = q2[u];
    __syncthreads();
    stamp(7);          // (diagnostic: k~ staged)
    // wave w: A2 rows p 2 S2R + w + 8 k, k < 2 S2R / 8 (the 8 waves split the 2 S2R rows evenly)
    constexpr int RW = S2R > 0 ? 2 * S2R / 8 : 1;
    static_assert(S2R == 0 || (2 * S2R) % 8 == 0, "fused A2 rows: a multiple of 8 rows per workgroup");
    sim2_wave_rows<RW>(kimg, kimg + S2_KIMG, wave, 8, lane, s2.a2, s2.a2s,
                       ((size_t)bh * NL + (size_t)p * 2 * S2R + wave) * NL, (size_t)8 * NL, (size_t)nbh * NL * NL);
  }
  const size_t pidx = ((size_t)p * nbh + bh) * NL + qi;
  if (h == 0) { part_m[pidx] = m_run; part_l[pidx] = l_run; }
  // the unnormalised partial sum in bf16 (half the slab bytes out and through the combine, which
  // merges the partials in fp32); m / l stay fp32
  bf16* po = part_o + pidx * DH;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
      *(bf16x4*)(po + dt * 32 + 8 * g4 + 4 * h) =
          (bf16x4){(bf16)o[dt][4 * g4], (bf16)o[dt][4 * g4 + 1], (bf16)o[dt][4 * g4 + 2], (bf16)o[dt][4 * g4 + 3]};
  if (ST) {
    __builtin_amdgcn_s_waitcnt(0);
    stamp(6);
  }
}

// combine of the v2 partials: grid (nbh, 32), block 256 (a3_combine.h; the bench step runs the same
// routine inside the pseudo-inverse chain's last launch instead, tm_pinv_fwd_split_a3)
__global__ __launch_bounds__(256) void a3_combine_v2_kernel(A3Combine c) {
  __shared__ A3CombineLds lds;
  const A3CombineState st = a3_combine_phase1(c, blockIdx.x, blockIdx.y, threadIdx.x, lds, true);
  __syncthreads();
  a3_combine_phase2(c, blockIdx.x, blockIdx.y, threadIdx.x, lds, st, true);
}

// combine the key-block partials: W[bh][q][d], lse3[bh][q]; grid (nbh, 16), block 256: thread =
// (query blockIdx.y * 16 + tid / 16, 4 consecutive d).  The partials of U key blocks are requested
// in one burst (clamped indices, masked adds), key blocks summed in index order.
constexpr int A3C_U = 11;
__global__ __launch_bounds__(256) void a3_combine_kernel(const float* __restrict__ part_o, const float* __restrict__ part_m,
                                                         const float* __restrict__ part_l, int nkb, int nbh,
                                                         float* __restrict__ w, float* __restrict__ lse3) {
  const int bh = blockIdx.x, qi = blockIdx.y * 16 + (threadIdx.x >> 4), d4 = (threadIdx.x & 15) * 4;
  const size_t q0 = (size_t)bh * NL + qi, kstride = (size_t)nbh * NL;
  float M = -INFINITY;
  for (int kb0 = 0; kb0 < nkb; kb0 += A3C_U) {
    float mv[A3C_U];
#pragma unroll
    for (int u = 0; u < A3C_U; ++u) mv[u] = part_m[(size_t)min(kb0 + u, nkb - 1) * kstride + q0];
#pragma unroll
    for (int u = 0; u < A3C_U; ++u) M = fmaxf(M, mv[u]);  // clamped repeats change nothing
  }
  float L = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int kb0 = 0; kb0 < nkb; kb0 += A3C_U) {
    float mv[A3C_U], lv[A3C_U];
    f32x4 ov[A3C_U];
#pragma unroll
    for (int u = 0; u < A3C_U; ++u) {
      const size_t pidx = (size_t)min(kb0 + u, nkb - 1) * kstride + q0;
      mv[u] = part_m[pidx];
      lv[u] = part_l[pidx];
      ov[u] = *(const f32x4*)(part_o + pidx * DH + d4);
    }
#pragma unroll
    for (int u = 0; u < A3C_U; ++u) {
      if (kb0 + u < nkb) {
        const float sc = __expf(mv[u] - M);
        L += lv[u] * sc;
        acc += ov[u] * sc;
      }
    }
  }
  *(f32x4*)(w + q0 * DH + d4) = acc / L;
  if (d4 == 0) lse3[q0] = M + __logf(L);
}

// ---------------------------------------------------------------------------
// D3[bh][q] = dW[q] . W[q]; dW_t = T(dW).  grid (nbh*256/4), block 256 (one wave per row)
template <typename T>
__global__ void rowdot_cast_kernel(const float* __restrict__ dw, const float* __restrict__ w, float* __restrict__ dd,
                                   T* __restrict__ dw_t, int rows) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float a = dw[(size_t)r * DH + lane];
  const float s = wave_sum(a * w[(size_t)r * DH + lane]);
  dw_t[(size_t)r * DH + lane] = from_f<T>(a);
  if (lane == 0) dd[r] = s;
}

// T copy of an fp32 [rows][64] matrix
template <typename T>
__global__ void cast_rows_kernel(const float* __restrict__ x, T* __restrict__ y, long long count) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i + 8 <= count) {
    store8<T>(y + i, cvt8<T>(x + i));
  } else {
    for (long long j = i; j < count; ++j) y[j] = from_f<T>(x[j]);
  }
}

// ---------------------------------------------------------------------------
// conv33 backward + D1.  grid (n/64, nbh), block 256.
//   dv[bh][t][d]  = sum_tau w[tau] dO[t - tau + 16][d]          (written, fp32)
//   c_tau(t)      = sum_d dO[t][d] v[t + tau - 16][d]
//   D1[bh][t]     = dO[t].O[t] - sum_tau w[tau] c_tau(t)          (= dO . (attn1 Y) )
//   dw_part[bag*ntb + tb][head*33 + tau] = sum_{t in block} c_tau(t)
// 96 staged rows (64 + 2*16 halo) of dO and v in fp32 LDS (272-B rows, b128 reads);
// a thread owns one row and every 4th tap, so each dO piece is read once per 9 taps.
template <typename T>
__global__ __launch_bounds__(256, 2) void conv_bwd_kernel(const T* __restrict__ dmerged, const T* __restrict__ merged,
                                                       const T* __restrict__ v, const float* __restrict__ wconv,
                                                       int n, int nh, T* __restrict__ dv, float* __restrict__ d1,
                                                       float* __restrict__ dw_part) {
  constexpr int R = 64, HR = R + 2 * HALF, RW = DH + 4;  // 96 staged rows, 68-float rows
  constexpr int NTQ = (TAPS + 3) / 4;                    // taps per thread (9)
  __shared__ __attribute__((aligned(16))) float dos[HR][RW];
  __shared__ __attribute__((aligned(16))) float vs[HR][RW];
  __shared__ float cred[R][TAPS + 1];
  __shared__ float ws[TAPS];
  const int bh = blockIdx.y, tb = blockIdx.x, tid = threadIdx.x;
  const int head = bh % nh, bag = bh / nh, ntb = gridDim.x;
  const int t0 = tb * R;
  const int ld = nh * DH;
  const T* dob = dmerged + (size_t)bag * n * ld + head * DH;
  const T* ob = merged + (size_t)bag * n * ld + head * DH;
  const T* vb = v + (size_t)bh * n * DH;
  constexpr int E = 16 / sizeof(T);
  constexpr int PER = HR * DH / E / 256;  // 16-B pieces per thread and tensor
  // one burst: the dO / v windows, this thread's quarter row of O and the conv taps
  Chunk16<T> ca[PER], cb[PER], co[16 / E];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + 256 * j, rr = i / (DH / E), d0 = (i % (DH / E)) * E, t = t0 - HALF + rr;
    if (t >= 0 && t < n) {
      ca[j].raw = *(const f32x4*)(dob + (size_t)t * ld + d0);
      cb[j].raw = *(const f32x4*)(vb + (size_t)t * DH + d0);
    } else {
      ca[j].raw = (f32x4){};
      cb[j].raw = (f32x4){};
    }
  }
  {
    const int t = t0 + (tid >> 2), dq0 = (tid & 3) * 16;
#pragma unroll
    for (int part = 0; part < 16 / E; ++part)
      co[part].raw = t < n ? *(const f32x4*)(ob + (size_t)t * ld + dq0 + part * E) : (f32x4){};
  }
  const float wtap = tid < TAPS ? wconv[head * TAPS + tid] : 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + 256 * j, rr = i / (DH / E), d0 = (i % (DH / E)) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      dos[rr][d0 + e] = to_f(ca[j].e[e]);
      vs[rr][d0 + e] = to_f(cb[j].e[e]);
    }
  }
  if (tid < TAPS) ws[tid] = wtap;
  __syncthreads();
  // part A: thread (row rl, tap phase qq): taps qq, qq+4, ...
  {
    const int rl = tid >> 2, qq = tid & 3, t = t0 + rl;
    float c[NTQ];
#pragma unroll
    for (int k = 0; k < NTQ; ++k) c[k] = 0.f;
    float dd = 0.f;
#pragma unroll
    for (int dc = 0; dc < DH; dc += 16) {
      float g[16];
#pragma unroll
      for (int e = 0; e < 16; e += 4) {
        const f32x4 x4 = *(const f32x4*)&dos[rl + HALF][dc + e];
        g[e] = x4[0]; g[e + 1] = x4[1]; g[e + 2] = x4[2]; g[e + 3] = x4[3];
      }
#pragma unroll
      for (int k = 0; k < NTQ; ++k) {
        const int tau = qq + 4 * k;
        if (tau < TAPS) {
#pragma unroll
          for (int e = 0; e < 16; e += 4) {
            const f32x4 x4 = *(const f32x4*)&vs[rl + tau][dc + e];
            c[k] = fmaf(g[e], x4[0], c[k]); c[k] = fmaf(g[e + 1], x4[1], c[k]);
            c[k] = fmaf(g[e + 2], x4[2], c[k]); c[k] = fmaf(g[e + 3], x4[3], c[k]);
          }
        }
      }
      if (dc / 16 == qq) {  // this thread's quarter of dO . O (co is zero past n)
#pragma unroll
        for (int part = 0; part < 16 / E; ++part)
#pragma unroll
          for (int e = 0; e < E; ++e) dd = fmaf(g[part * E + e], to_f(co[part].e[e]), dd);
      }
    }
    float wc = 0.f;
#pragma unroll
    for (int k = 0; k < NTQ; ++k) {
      const int tau = qq + 4 * k;
      if (tau < TAPS) { cred[rl][tau] = c[k]; wc = fmaf(ws[tau], c[k], wc); }
    }
    float tot = dd - wc;
    tot += __shfl_xor(tot, 1, 64);
    tot += __shfl_xor(tot, 2, 64);
    if (qq == 0 && t < n) d1[(size_t)bh * n + t] = tot;
  }
  __syncthreads();
  if (tid < TAPS) {
    float sum = 0.f;
    for (int rl = 0; rl < R; ++rl) sum += cred[rl][tid];
    dw_part[((size_t)bag * ntb + tb) * (nh * TAPS) + head * TAPS + tid] = sum;
  }
  // part B: dv, thread (row rl, 16 d)
  {
    const int rl = tid >> 2, d0 = (tid & 3) * 16, t = t0 + rl;
    if (t < n) {
      float acc[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll 3
      for (int tau = 0; tau < TAPS; ++tau) {
        const float wt = ws[tau];
#pragma unroll
        for (int e = 0; e < 16; e += 4) {
          const f32x4 x4 = *(const f32x4*)&dos[rl + 2 * HALF - tau][d0 + e];
          acc[e] = fmaf(wt, x4[0], acc[e]); acc[e + 1] = fmaf(wt, x4[1], acc[e + 1]);
          acc[e + 2] = fmaf(wt, x4[2], acc[e + 2]); acc[e + 3] = fmaf(wt, x4[3], acc[e + 3]);
        }
      }
      T* dst = dv + ((size_t)bh * n + t) * DH + d0;   // dv in the step's dtype
#pragma unroll
      for (int e = 0; e < 16; ++e) dst[e] = from_f<T>(acc[e]);
    }
  }
}

// ---------------------------------------------------------------------------
// bf16 conv33 backward on the MFMA.  One workgroup = one head x R rows, R = n * nbh / 256
// rounded up to 8 (<= 288): 256 workgroups at N = 8192 (the fp32-LDS kernel above runs 1056
// workgroups of 64 rows, three rounds deep, bound by its LDS reads: 30 us).  Windows of 320
// rows (t0 - 16 ..) of dO and v as bf16 row-major LDS images; per 32-row tile i (wave w takes
// tiles w, w + 8):
//   S  = dO[tile] v_win[32i .. 32i + 63]^T (2 MFMA tiles, K = 64)  ->  c_tau(t) = S[r][r + tau]
//   dv = Toep(w) dO_win[32i .. 32i + 63],  Toep[r][k] = w[r + 32 - k]  (w as bf16 hi + lo, so
//        the taps keep ~16 bits; the products of bf16 operands are exact in the fp32 sums)
constexpr int CB_ROWS = 288, CB_WIN = CB_ROWS + 2 * HALF, CB_ROW = DH + 8, CB_ST = 66;
struct CbLay {
  static constexpr size_t DO_OFF = 0;
  static constexpr size_t V_OFF = DO_OFF + (size_t)CB_WIN * CB_ROW * 2;
  static constexpr size_t ST_OFF = V_OFF + (size_t)CB_WIN * CB_ROW * 2;  // [8 waves][32][66] fp32
  static constexpr size_t W_OFF = ST_OFF + 8 * 32 * CB_ST * 4;            // taps fp32
  static constexpr size_t CS_OFF = W_OFF + 64 * 4;                        // [8 waves][36] tap sums
  static constexpr size_t BYTES = CS_OFF + 8 * 36 * 4;                    // 161152
};

// rows per workgroup of the bf16 conv backward (one workgroup per CU over all heads when possible)
inline int conv_bwd_rows(int nbh, int n) {
  const long long cu = tm_cu_count();
  const long long want = ((long long)n * nbh + cu - 1) / cu;
  const int r = (int)((want + 7) / 8 * 8);
  return r < 32 ? 32 : (r > CB_ROWS ? CB_ROWS : r);
}

// standard B fragment (lane: col = mb + (lane & 31), k = kb + 8 (lane >> 5) + j) of a row-major
// [k][ldr] bf16 LDS image, by two transposing reads
TM_DEV bf16x8 frag_tr_rows(const bf16* S, int ldr, int mb, int kb, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int m = mb + (g & 1) * 16 + 4 * p;
  const int k = kb + 8 * (g >> 1) + q;
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(S + k * ldr + m));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(S + (k + 4) * ldr + m));
  return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__global__ __launch_bounds__(512) void conv_bwd_mfma_kernel(const bf16* __restrict__ dmerged,
                                                            const bf16* __restrict__ merged,
                                                            const bf16* __restrict__ v,
                                                            const float* __restrict__ wconv, int n, int nh, int R,
                                                            bf16* __restrict__ dv, float* __restrict__ d1,
                                                            float* __restrict__ dw_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* dos = (bf16*)(smem + CbLay::DO_OFF);
  bf16* vws = (bf16*)(smem + CbLay::V_OFF);
  float* ws = (float*)(smem + CbLay::W_OFF);
  float* csum = (float*)(smem + CbLay::CS_OFF);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int bh = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
  const int head = bh % nh, bag = bh / nh, ld = nh * DH;
  const int t0 = blk * R;
  const int rows = min(R, n - t0);
  const bf16* dob = dmerged + (size_t)bag * n * ld + head * DH;
  const bf16* ob = merged + (size_t)bag * n * ld + head * DH;
  const bf16* vb = v + (size_t)bh * n * DH;
  // the two windows in one burst (rows past what the block's tiles read stay zero)
  constexpr int PW = CB_WIN * 8 / 512;
  bf16x8 ca[PW], cb[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int i = tid + 512 * j, w = i >> 3, d0 = (i & 7) * 8, t = t0 - HALF + w;
    const bool ok = t >= 0 && t < n && w < rows + 2 * HALF;
    const int tc = ok ? t : 0;
    ca[j] = load8(dob + (size_t)tc * ld + d0);
    cb[j] = load8(vb + (size_t)tc * DH + d0);
    if (!ok) { ca[j] = (bf16x8){}; cb[j] = (bf16x8){}; }
  }
  if (tid < TAPS) ws[tid] = wconv[head * TAPS + tid];
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int i = tid + 512 * j, w = i >> 3, d0 = (i & 7) * 8;
    *(bf16x8*)(dos + w * CB_ROW + d0) = ca[j];
    *(bf16x8*)(vws + w * CB_ROW + d0) = cb[j];
  }
  __syncthreads();
  // Toeplitz A fragments (the same for every tile): lane row r32, k = 16 s + 8 h + j
  bf16x8 th[4], tl[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int tau = r32 + 32 - (16 * st + 8 * h + j);
      const float wv = (tau >= 0 && tau < TAPS) ? ws[tau] : 0.f;
      const bf16 hi = (bf16)wv;
      th[st][j] = hi;
      tl[st][j] = (bf16)(wv - (float)hi);
    }
  }
  float* stg = (float*)(smem + CbLay::ST_OFF) + wave * 32 * CB_ST;
  constexpr int NTK = (TAPS + 1) / 2;  // taps per lane: tau = h + 2k (17)
  float csl[NTK];
#pragma unroll
  for (int k = 0; k < NTK; ++k) csl[k] = 0.f;
  const int ntile = (rows + 31) / 32;
#pragma unroll 1
  for (int i = wave; i < ntile; i += 8) {
    // S = dO[tile] . v_win[32i .. 32i + 63]^T
    f32x16 sa = (f32x16){}, sb = (f32x16){};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const bf16x8 a = *(const bf16x8*)(dos + (32 * i + HALF + r32) * CB_ROW + 16 * st + 8 * h);
      const bf16x8 ba = *(const bf16x8*)(vws + (32 * i + r32) * CB_ROW + 16 * st + 8 * h);
      const bf16x8 bb = *(const bf16x8*)(vws + (32 * i + 32 + r32) * CB_ROW + 16 * st + 8 * h);
      mma16(sa, a, ba);
      mma16(sb, a, bb);
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = acc_row(reg, h);
      stg[row * CB_ST + r32] = sa[reg];
      stg[row * CB_ST + 32 + r32] = sb[reg];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // band: lane (row r32, taps h + 2k); the row's dO . O over d 32h .. 32h + 31
    const int lr = 32 * i + r32;
    const bool rv = lr < rows;
    float wc = 0.f, dd = 0.f;
#pragma unroll
    for (int k = 0; k < NTK; ++k) {
      const int tau = h + 2 * k;
      if (tau < TAPS) {
        const float c = stg[r32 * CB_ST + r32 + tau];
        if (rv) { csl[k] += c; wc = fmaf(ws[tau], c, wc); }
      }
    }
    if (rv) {
      const bf16* orow = ob + (size_t)(t0 + lr) * ld + 32 * h;
      const bf16* grow = dos + (lr + HALF) * CB_ROW + 32 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bf16x8 o8 = load8(orow + 8 * q), g8 = *(const bf16x8*)(grow + 8 * q);
#pragma unroll
        for (int e = 0; e < 8; ++e) dd = fmaf((float)g8[e], (float)o8[e], dd);
      }
    }
    float tot = dd - wc;
    tot += __shfl_xor(tot, 32, 64);
    if (rv && h == 0) d1[(size_t)bh * n + t0 + lr] = tot;
    // dv tile = Toep . dO_win[32i .. 32i + 63]
    const bf16* dwin = dos + 32 * i * CB_ROW;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      f32x16 acc = (f32x16){};
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const bf16x8 b = frag_tr_rows(dwin, CB_ROW, dt * 32, 16 * st, lane);
        mma16(acc, th[st], b);
        mma16(acc, tl[st], b);
      }
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int l2 = 32 * i + acc_row(reg, h);
        if (l2 < rows) dv[((size_t)bh * n + t0 + l2) * DH + dt * 32 + r32] = (bf16)acc[reg];   // bf16: read once by the fused A3 backward
      }
    }
    __builtin_amdgcn_wave_barrier();   // the stage is rewritten by the wave's next tile
  }
  // tap sums: over the 32 rows of each lane half, then over the waves in a fixed order
#pragma unroll
  for (int k = 0; k < NTK; ++k) {
    float x = csl[k];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) x += __shfl_xor(x, o, 64);
    const int tau = h + 2 * k;
    if (r32 == 0 && tau < TAPS) csum[wave * 36 + tau] = x;
  }
  __syncthreads();
  if (tid < TAPS) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) sum += csum[w * 36 + tid];
    dw_part[((size_t)bag * nblk + blk) * (nh * TAPS) + head * TAPS + tid] = sum;
  }
}

// ---------------------------------------------------------------------------
// Flash-style backward shared by both attention products.  A workgroup owns a
// block of 256 keys (4 waves x 64, key on the MFMA lane) and walks query chunks
// of 32.  With P = exp(Q K^T - lse), dS = P (dO V^T - D):
//   dV^T += dO^T P,  dK^T += Q^T dS   (registers, sum over the walked queries)
//   dQ    = dS K                      (per chunk, dS through LDS)
// MODE_A3: keys = k rows (block kb), queries = all 256 landmarks;
//          dK -> dk (=), dV -> dv (+=), dQ -> partial slab [kb] (dql).
// MODE_A1: keys = the 256 landmarks, queries = rows [qc*QC, (qc+1)*QC);
//          dQ -> dq (=), dK -> partial slab [qc] (dkl), dV -> partial slab [qc] (dY).
struct BwdArgs {
  const void* q; long long q_bag, q_head; int q_row;    // queries (T)
  const void* dO; long long o_bag, o_head; int o_row;   // upstream grad (T)
  const void* k; long long k_bag, k_head;               // keys (T), row stride 64
  const void* v; long long v_bag, v_head;               // values (T), row stride 64
  const float* lse;  long long lse_bh;                  // [bh][...]
  const float* dd;   long long dd_bh;                   // D per query
  const float* dd2;                                     // optional second partial of D (summed: dd + dd2)
  float* dq; long long dq_bh;                           // query-side grad (fp32, row stride 64)
  float* dk; long long dk_bh;                           // key-side grads (fp32, row stride 64)
  float* dv; long long dv_bh;
  long long slab_stride;                                // per block partial slab stride (MODE dependent)
  int nh, n_queries_per_wg, n_key_rows;
  int q_total;  // bf16 A1 kernel: > 0 = split the q_total / 32 query chunks evenly over gridDim.x
  // bf16 A3 kernel, fused key side: non-null = write the FINAL k / v parts of dqkv (bf16,
  // [bag][n][3 nh 64]): k = dK + dk~[t / l] / l, v = dv (the conv backward's, read) + dV
  void* dqkv; const float* dkl; float inv_l; int l;
  int dv_lo, dv_hi;   // fused: rows of the conv backward's dv that are read (zero outside)
  // bf16 A1 kernel: dqkv non-null = dq written as bf16(dq_scale * dq) into the q part of dqkv
  // ([bag][q_total][3 nh 64], the columns of head bh % nh) instead of fp32 rows at dq
  float dq_scale;
  // 1 = partial slabs written as bf16 (half the slab bytes out and back; their consumers sum them in
  // fp32): the bf16 A1 kernel's dk~ / dY slabs (through the deferred flush), the fused A3 backward's
  // dq~ slab (through assemble_q_slab / cls_q_rows); the slab strides then count bf16 elements
  int slab_bf16;
};

enum { MODE_A3 = 0, MODE_A1 = 1 };
}  // namespace
// gemm.hip (library-internal): split-K sum of fp32 or bf16 partial slabs, deferred into q when given
int tm_splitk_reduce_typed(const void* slab, int slab_dtype, float* out, int splits, long long count, float alpha,
                           int accumulate, tm_reduce_queue* q, void* stream);
namespace {
#ifdef TM_DIAG
int g_nys_variant = 0;
#endif
#define NYS_VARIANT TM_DIAG_VAR(g_nys_variant)

template <typename T> struct BwdLay {
  static constexpr int QT_ROW = 32 + 4;              // Q^T / dO^T chunk [64 d][36]
  static constexpr int KT_ROW = NL + 16 / sizeof(T); // K^T [64 d][264 bf16 / 260 f32]
  static constexpr int DS_ROW = KT_ROW;              // dS  [32 q][...]
  static constexpr size_t KT_OFF = 0;
  static constexpr size_t DS_OFF = KT_OFF + DH * KT_ROW * sizeof(T);
  static constexpr size_t QT_OFF = DS_OFF + 32 * DS_ROW * sizeof(T);
  static constexpr size_t OT_OFF = QT_OFF + DH * QT_ROW * sizeof(T);
  static constexpr size_t XC_OFF = OT_OFF + DH * QT_ROW * sizeof(T);   // fp32 [3][2][1024]
  static constexpr size_t LS_OFF = XC_OFF + 6 * 1024 * 4;              // fp32 lse[32], D[32]
  static constexpr size_t MAIN = LS_OFF + 64 * 4;
  static constexpr size_t EPI = (size_t)NL * 68 * 4;                   // key-side transpose stage
  static constexpr size_t BYTES = MAIN > EPI ? MAIN : EPI;
};

// 8 waves x 32 keys.  The wave's K and V fragments stay in registers for the
// whole query walk; per 32-query chunk: S, dP (8 MFMAs), dV^T, dK^T (8 MFMAs),
// and a quarter of dQ = dS K (4 MFMAs) reduced across the 4 key quarters in LDS.
template <typename T, int MODE>
__global__ __launch_bounds__(512) void attn_bwd_kernel(BwdArgs a) {
  using LY = BwdLay<T>;
  constexpr int QT_ROW = LY::QT_ROW, KT_ROW = LY::KT_ROW, DS_ROW = LY::DS_ROW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* kt_s = (T*)(smem + LY::KT_OFF);
  T* ds_s = (T*)(smem + LY::DS_OFF);
  T* qt_s = (T*)(smem + LY::QT_OFF);
  T* dot_s = (T*)(smem + LY::OT_OFF);
  float* xch = (float*)(smem + LY::XC_OFF);
  float* lse_s = (float*)(smem + LY::LS_OFF);
  float* dd_s = lse_s + 32;
  float* stage = (float*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int blk = blockIdx.x, bh = blockIdx.y, nh = a.nh;
  const int key0 = (MODE == MODE_A3) ? blk * NL : 0;
  const int q_begin = (MODE == MODE_A1) ? blk * a.n_queries_per_wg : 0;
  const int q_count = a.n_queries_per_wg;

  const T* Q = (const T*)a.q + hoff(bh, nh, a.q_bag, a.q_head);
  const T* dO = (const T*)a.dO + hoff(bh, nh, a.o_bag, a.o_head);
  const T* K = (const T*)a.k + hoff(bh, nh, a.k_bag, a.k_head) + (size_t)key0 * DH;
  const T* V = (const T*)a.v + hoff(bh, nh, a.v_bag, a.v_head) + (size_t)key0 * DH;
  const float* lse = a.lse + bh * a.lse_bh;
  const float* dd = a.dd + bh * a.dd_bh;
  const float* dd2 = a.dd2 ? a.dd2 + bh * a.dd_bh : nullptr;

  // K^T into LDS (all 256 keys): 16-B row loads, transposed element writes
  {
    constexpr int E = 16 / sizeof(T);
    for (int c = tid; c < NL * DH / E; c += 512) {
      const int key = c / (DH / E), d0 = (c % (DH / E)) * E;
      const vec8<T> v8 = E == 8 ? load8(K + (size_t)key * DH + d0) : vec8<T>{};
      if constexpr (E == 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) kt_s[(d0 + e) * KT_ROW + key] = v8[e];
      } else {
        const vec4<T> v4 = load4(K + (size_t)key * DH + d0);
#pragma unroll
        for (int e = 0; e < 4; ++e) kt_s[(d0 + e) * KT_ROW + key] = v4[e];
      }
    }
  }
  const int mykey = wave * 32;
  vec8<T> kf[4], vf[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    kf[st] = load8(K + (size_t)(mykey + r) * DH + st * 16 + 8 * h);
    vf[st] = load8(V + (size_t)(mykey + r) * DH + st * 16 + 8 * h);
  }

  f32x16 dvt[2], dkt[2];  // [d tile], cols = this wave's 32 keys
#pragma unroll
  for (int i = 0; i < 2; ++i) { dvt[i] = (f32x16){}; dkt[i] = (f32x16){}; }

  const int dt_q = wave & 1, kq = wave >> 1;  // dQ role: d tile, key quarter
#pragma unroll 1
  for (int c0 = 0; c0 < q_count; c0 += 32) {
    const int qa = q_begin + c0;
    __syncthreads();  // previous chunk fully consumed
    {
      // one 16-B row piece per thread: threads 0..255 Q, 256..511 dO (bf16: 8 d each)
      constexpr int E = 16 / sizeof(T);
      const int which = tid >> 8, c = tid & 255;
      const T* src = which ? dO : Q;
      const int row = which ? a.o_row : a.q_row;
      T* dst = which ? dot_s : qt_s;
      for (int cc = c; cc < 32 * DH / E; cc += 256) {
        const int qq = cc / (DH / E), d0 = (cc % (DH / E)) * E;
        if constexpr (E == 8) {
          const vec8<T> v8 = load8(src + (size_t)(qa + qq) * row + d0);
#pragma unroll
          for (int e = 0; e < 8; ++e) dst[(d0 + e) * QT_ROW + qq] = v8[e];
        } else {
          const vec4<T> v4 = load4(src + (size_t)(qa + qq) * row + d0);
#pragma unroll
          for (int e = 0; e < 4; ++e) dst[(d0 + e) * QT_ROW + qq] = v4[e];
        }
      }
    }
    if (tid < 32) { lse_s[tid] = lse[qa + tid]; dd_s[tid] = dd[qa + tid] + (dd2 ? dd2[qa + tid] : 0.f); }
    __syncthreads();
    // S = Q K^T, dP = dO V^T: rows = queries (registers), cols = this wave's keys (lanes)
    f32x16 s = (f32x16){}, dp = (f32x16){};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const vec8<T> qa_f = load8(Q + (size_t)(qa + r) * a.q_row + st * 16 + 8 * h);
      const vec8<T> oa_f = load8(dO + (size_t)(qa + r) * a.o_row + st * 16 + 8 * h);
      mma16(s, qa_f, kf[st]);
      mma16(dp, oa_f, vf[st]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qq = acc_row(i, h);
      const float p = __expf(s[i] - lse_s[qq]);
      s[i] = p;
      dp[i] = p * (dp[i] - dd_s[qq]);
    }
    // dV^T += dO^T P ; dK^T += Q^T dS
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      const vec8<T> bp = acc_as_operand<T>(s, sp);
      const vec8<T> bs = acc_as_operand<T>(dp, sp);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const T* ro = dot_s + (dt * 32 + r) * QT_ROW + 16 * sp + 4 * h;
        const T* rq = qt_s + (dt * 32 + r) * QT_ROW + 16 * sp + 4 * h;
        const vec4<T> o0 = load4(ro), o1 = load4(ro + 8), q0 = load4(rq), q1 = load4(rq + 8);
        vec8<T> ao, aq;
#pragma unroll
        for (int e = 0; e < 4; ++e) { ao[e] = o0[e]; ao[4 + e] = o1[e]; aq[e] = q0[e]; aq[4 + e] = q1[e]; }
        mma16(dvt[dt], ao, bp);
        mma16(dkt[dt], aq, bs);
      }
    }
    // dS -> LDS [q][key]
#pragma unroll
    for (int i = 0; i < 16; ++i) ds_s[acc_row(i, h) * DS_ROW + mykey + r] = from_f<T>(dp[i]);
    __syncthreads();
    // dQ chunk [32 q x 64 d] = dS [32 x 256] . K [256 x 64]: this wave: d tile dt_q, keys 64*kq..+63
    {
      f32x16 acc = (f32x16){};
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int kk = kq * 64 + st * 16 + 8 * h;
        mma16(acc, load8(ds_s + r * DS_ROW + kk), load8(kt_s + (dt_q * 32 + r) * KT_ROW + kk));
      }
      if (kq > 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) xch[((kq - 1) * 2 + dt_q) * 1024 + i * 64 + lane] = acc[i];
      }
      __syncthreads();
      if (kq == 0) {
        float* dst;
        if (MODE == MODE_A1) dst = a.dq + bh * a.dq_bh;
        else dst = a.dq + (size_t)blk * a.slab_stride + bh * a.dq_bh;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qq = qa + acc_row(i, h);
          const float v = ((acc[i] + xch[(0 * 2 + dt_q) * 1024 + i * 64 + lane]) +
                           xch[(1 * 2 + dt_q) * 1024 + i * 64 + lane]) + xch[(2 * 2 + dt_q) * 1024 + i * 64 + lane];
          dst[(size_t)qq * DH + dt_q * 32 + r] = v;
        }
      }
    }
  }
  // ---- key-side epilogue through LDS (transpose to [key][d]) ----
  __syncthreads();
#pragma unroll
  for (int which = 0; which < 2; ++which) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const f32x16& accv = which == 0 ? dvt[dt] : dkt[dt];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        // registers 4g4..4g4+3 hold d = dt*32 + 8*g4 + 4h + 0..3 for key mykey + r
        *(f32x4*)(stage + (mykey + r) * 68 + dt * 32 + 8 * g4 + 4 * h) =
            (f32x4){accv[4 * g4], accv[4 * g4 + 1], accv[4 * g4 + 2], accv[4 * g4 + 3]};
      }
    }
    __syncthreads();
    if (MODE == MODE_A3 && a.dqkv) {
      // fused: the final bf16 k / v rows of dqkv (no fp32 key-side slabs, no assemble pass for them)
      const int bag = bh / nh, hh = bh % nh, inner = nh * DH;
      bf16* out = (bf16*)a.dqkv + ((size_t)bag * a.n_key_rows + key0) * 3 * inner + (which == 0 ? 2 : 1) * inner + hh * DH;
      const float* dvc = a.dv + bh * a.dv_bh + (size_t)key0 * DH;
      const float* dkl = a.dkl + (size_t)bh * NL * DH;
      for (int i = tid; i < NL * DH / 4; i += 512) {
        const int key = i >> 4, d4 = (i & 15) * 4;
        f32x4 val = *(const f32x4*)(stage + key * 68 + d4);
        if (which == 0) {
          if (key0 + key >= a.dv_lo && key0 + key < a.dv_hi) val += *(const f32x4*)(dvc + (size_t)key * DH + d4);
        }
        else val += *(const f32x4*)(dkl + (size_t)((key0 + key) / a.l) * DH + d4) * a.inv_l;
        *(bf16x4*)(out + (size_t)key * 3 * inner + d4) =
            (bf16x4){(bf16)val[0], (bf16)val[1], (bf16)val[2], (bf16)val[3]};
      }
      __syncthreads();
      continue;
    }
    float* dst;
    bool add = false;
    if (MODE == MODE_A3) {
      dst = (which == 0 ? a.dv + bh * a.dv_bh : a.dk + bh * a.dk_bh) + (size_t)key0 * DH;
      add = (which == 0);
    } else {
      dst = (which == 0 ? a.dv : a.dk) + (size_t)blk * a.slab_stride + bh * (which == 0 ? a.dv_bh : a.dk_bh);
    }
    for (int i = tid; i < NL * DH / 4; i += 512) {
      const int key = i >> 4, d4 = (i & 15) * 4;
      f32x4 val = *(const f32x4*)(stage + key * 68 + d4);
      float* p = dst + (size_t)key * DH + d4;
      if (add) val += *(const f32x4*)p;
      *(f32x4*)p = val;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// bf16 attention backward with every operand of the workgroup staged ONCE: the
// workgroup's <= 256 query rows of Q and dO ([q][72] row-major images), their lse / D,
// K^T and the wave's K / V fragments are all requested in one burst before the query
// walk, so the walk itself issues no global loads (the per-chunk version paid two
// dependent HBM round trips per 32-query chunk).  dV/dK operands come from the same
// row-major images through transposing reads (acc_as_operand k order).
// NW waves = NW 32-key units per workgroup; MQ = staged query rows.  <8, 288>: A1 (the 256
// landmark keys, <= 9 query chunks) and the A3 key blocks of 256; <9, 256>: A3 with the n / 32 key
// units of a head split evenly over 256 / nbh workgroups (8-9 units each: one chip round at
// N = 8192 where 33 blocks of 256 keys per head were 264 workgroups on 256 CUs).
template <int NW, int MQ>
struct BwdLayT {
  static constexpr int MAXQ = MQ;
  static constexpr int NK = 32 * NW;  // key columns
  static constexpr int KT_ROW = NK + 8, DS_ROW = NK + 8, QROW = DH + 8;
  static constexpr size_t KT_OFF = 0;
  static constexpr size_t DS_OFF = KT_OFF + DH * KT_ROW * 2;
  static constexpr size_t QS_OFF = DS_OFF + 32 * DS_ROW * 2;
  static constexpr size_t OS_OFF = QS_OFF + MAXQ * QROW * 2;
  static constexpr size_t XC_OFF = OS_OFF + MAXQ * QROW * 2;  // fp32 [3][32 q][64 d] key-group dq partials
  static constexpr size_t LS_OFF = XC_OFF + 6 * 1024 * 4;     // fp32 lse[MAXQ], D[MAXQ]
  static constexpr size_t MAIN = LS_OFF + 2 * MAXQ * 4;       // 160512 B (<8, 288>), 157184 B (<9, 256>)
  static constexpr size_t EPI = (size_t)NK * 68 * 4;
  static constexpr size_t BYTES = MAIN > EPI ? MAIN : EPI;
};
using BwdLay16 = BwdLayT<8, 288>;
using BwdLay9 = BwdLayT<9, 256>;
static_assert(BwdLay9::BYTES <= 160 * 1024 && BwdLay16::BYTES <= 160 * 1024, "bf16 backward layout exceeds the CU's LDS");

// A-operand fragment (rows m = mb + l32, 8 k in acc_as_operand order) of a row-major
// [k][QROW] bf16 image: element j of lane half h <-> k = kb + 8 (j >> 2) + 4 h + (j & 3)
template <int R>
TM_DEV bf16x8 frag_tr_rows(const bf16* S, int mb, int kb, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int m = mb + (g & 1) * 16 + 4 * p;
  const int k = kb + 4 * (g >> 1) + q;
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(S + k * R + m));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(S + (k + 8) * R + m));
  return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
TM_DEV bf16x8 frag_tr_acc(const bf16* S, int mb, int kb, int lane) { return frag_tr_rows<BwdLay16::QROW>(S, mb, kb, lane); }

// DQ2 (default): dQ = dS K by two waves, one 32-column d tile each over ALL the workgroup's keys in
// one accumulation chain (no cross-wave partials through LDS, no third barrier per chunk; the other
// waves go on to the next chunk's S / dP / dV / dK meanwhile).  DQ2 = 0: the earlier form (every
// wave a key group's partial, summed through LDS by the group-0 waves; diagnostic build only).
template <int MODE, int NW = 8, int ST = 0, int DQ2 = 1>   // ST: diagnostic s_memtime stamps (g_a1_stamps): 1 phases, 2 one chunk
                                                           // DQ2 = 2: the DQ2 chain with its reads just in time
__global__ __launch_bounds__(64 * NW) void attn_bwd_bf16_kernel(BwdArgs a) {
  using LY = std::conditional_t<NW == 9, BwdLay9, BwdLay16>;
  static_assert(NW == 8 || (NW == 9 && MODE == MODE_A3), "9-wave form: A3 even split only");
  constexpr int NT = 64 * NW;
  constexpr int KT_ROW = LY::KT_ROW, DS_ROW = LY::DS_ROW, QROW = LY::QROW;
  // dQ roles: 2 d tiles x NKQ key groups of KQS 16-deep k-steps (8 waves: 4 x 64 keys; 9: 3 x 96)
  constexpr int NKQ = NW == 9 ? 3 : 4, KQS = 2 * NW / NKQ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* kt_s = (bf16*)(smem + LY::KT_OFF);
  bf16* ds_s = (bf16*)(smem + LY::DS_OFF);
  bf16* qs = (bf16*)(smem + LY::QS_OFF);
  bf16* os = (bf16*)(smem + LY::OS_OFF);
  float* xch = (float*)(smem + LY::XC_OFF);
  float* lse_s = (float*)(smem + LY::LS_OFF);
  float* dd_s = lse_s + LY::MAXQ;
  float* stage = (float*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int blk = blockIdx.x, bh = blockIdx.y, nh = a.nh;
  auto stamp = [&](int slot) { if (ST == 1 && wave < 8) a1p_stamp<ST ? 9 : 0>(slot, wave); };
  auto cstamp = [&](int c0, int slot) { if (ST == 2 && c0 == 64 && wave < 8) a1p_stamp<ST ? 9 : 0>(slot, wave); };
  stamp(0);
  int key0 = (MODE == MODE_A3) ? blk * NL : 0;
  int nunits = 8;  // 32-key units of this workgroup (wave w < nunits owns keys key0 + 32 w ..)
  if (MODE == MODE_A3 && a.q_total > 0) {
    // even split of the head's n / 32 key units over the gridDim.x workgroups (<= NW each, host-checked)
    const int upk = a.n_key_rows / 32;
    const int u0 = (int)((long long)blk * upk / gridDim.x), u1 = (int)((long long)(blk + 1) * upk / gridDim.x);
    key0 = 32 * u0;
    nunits = u1 - u0;
  }
  const int nk = 32 * nunits;
  const bool active = wave < nunits;
  int q_begin = (MODE == MODE_A1) ? blk * a.n_queries_per_wg : 0;
  int q_count = a.n_queries_per_wg;  // <= 256, a multiple of 32 (host-checked)
  if (MODE == MODE_A1 && a.q_total > 0) {
    // even split of the q_total / 32 query chunks over the gridDim.x workgroups of a head: at
    // N = 8192 that is 8-9 chunks for each of 32 workgroups (256 = one per CU) instead of 33
    // blocks of 8 chunks (264 > 256 CUs: a second round for 8 of them)
    const int cph = a.q_total / 32;
    const int c0 = (int)((long long)blk * cph / gridDim.x), c1 = (int)((long long)(blk + 1) * cph / gridDim.x);
    q_begin = 32 * c0;
    q_count = 32 * (c1 - c0);  // <= MAXQ (host-checked)
  }

  const bf16* Q = (const bf16*)a.q + hoff(bh, nh, a.q_bag, a.q_head) + (size_t)q_begin * a.q_row;
  const bf16* dO = (const bf16*)a.dO + hoff(bh, nh, a.o_bag, a.o_head) + (size_t)q_begin * a.o_row;
  const bf16* K = (const bf16*)a.k + hoff(bh, nh, a.k_bag, a.k_head) + (size_t)key0 * DH;
  const bf16* V = (const bf16*)a.v + hoff(bh, nh, a.v_bag, a.v_head) + (size_t)key0 * DH;
  const float* lse = a.lse + bh * a.lse_bh + q_begin;
  const float* dd = a.dd + bh * a.dd_bh + q_begin;
  const float* dd2 = a.dd2 ? a.dd2 + bh * a.dd_bh + q_begin : nullptr;

  // ---- one burst of loads: K rows (for K^T), Q / dO rows, K / V fragments, lse / D ----
  constexpr int QP = (LY::MAXQ * 8 + NT - 1) / NT;  // 16-B query-row pieces per thread (5 | 4)
  const int mykey = wave * 32;
  bf16x8 qr[QP], orow[QP], kf[4], vf[4];
  // key rows past nk (a short workgroup of the even split): clamped loads, finite, and their dS
  // columns are written as zeros, so they add nothing to dQ.  K^T is staged from the waves' own K
  // fragments (no second read of the K rows)
#pragma unroll
  for (int j = 0; j < QP; ++j) {
    const int c = tid + NT * j;
    const int qq = min(c >> 3, q_count - 1);  // rows past q_count: clamped, never read back
    qr[j] = load8(Q + (size_t)qq * a.q_row + (c & 7) * 8);
    orow[j] = load8(dO + (size_t)qq * a.o_row + (c & 7) * 8);
  }
  const int kfr = min(mykey + r, nk - 1);
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    kf[st] = load8(K + (size_t)kfr * DH + st * 16 + 8 * h);
    vf[st] = load8(V + (size_t)kfr * DH + st * 16 + 8 * h);
  }
  float lsev = 0.f, ddv = 0.f;
  if (tid < LY::MAXQ) {
    const int qq = min(tid, q_count - 1);
    lsev = lse[qq];
    ddv = dd[qq] + (dd2 ? dd2[qq] : 0.f);
  }
  __builtin_amdgcn_sched_barrier(0);
  stamp(1);
#pragma unroll
  for (int st = 0; st < 4; ++st) {   // this lane's key mykey + r, d = 16 st + 8 h .. + 7
#pragma unroll
    for (int e = 0; e < 8; ++e) kt_s[(st * 16 + 8 * h + e) * KT_ROW + mykey + r] = kf[st][e];
  }
#pragma unroll
  for (int j = 0; j < QP; ++j) {
    const int c = tid + NT * j, row = c >> 3, d0 = (c & 7) * 8;
    if (row < LY::MAXQ) {
      *(bf16x8*)(qs + row * QROW + d0) = qr[j];
      *(bf16x8*)(os + row * QROW + d0) = orow[j];
    }
  }
  if (tid < LY::MAXQ) {
    lse_s[tid] = lsev;
    dd_s[tid] = ddv;
  }
  __syncthreads();
  stamp(2);

  f32x16 dvt[2], dkt[2];  // [d tile], cols = this wave's 32 keys
#pragma unroll
  for (int i = 0; i < 2; ++i) { dvt[i] = (f32x16){}; dkt[i] = (f32x16){}; }

  const int dt_q = wave & 1, kq = wave >> 1;  // dQ role: d tile, key group (waves < 2 NKQ)
  const bool dq_role = wave < 2 * NKQ;
#pragma unroll 1
  for (int c0 = 0; c0 < q_count; c0 += 32) {
    // S = Q K^T, dP = dO V^T: rows = queries (registers), cols = this wave's keys (lanes)
    f32x16 s = (f32x16){}, dp = (f32x16){};
    cstamp(c0, 0);
    if (active) {
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const bf16x8 qa_f = *(const bf16x8*)(qs + (c0 + r) * QROW + st * 16 + 8 * h);
        const bf16x8 oa_f = *(const bf16x8*)(os + (c0 + r) * QROW + st * 16 + 8 * h);
        mma16(s, qa_f, kf[st]);
        mma16(dp, oa_f, vf[st]);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qq = c0 + acc_row(i, h);
        const float p = __expf(s[i] - lse_s[qq]);
        s[i] = p;
        dp[i] = p * (dp[i] - dd_s[qq]);
      }
      // dV^T += dO^T P ; dK^T += Q^T dS
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const bf16x8 bp = acc_as_operand<bf16>(s, sp);
        const bf16x8 bs = acc_as_operand<bf16>(dp, sp);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16x8 ao = frag_tr_acc(os + c0 * QROW, dt * 32, 16 * sp, lane);
          const bf16x8 aq = frag_tr_acc(qs + c0 * QROW, dt * 32, 16 * sp, lane);
          mma16(dvt[dt], ao, bp);
          mma16(dkt[dt], aq, bs);
        }
      }
    }
    cstamp(c0, 1);
    __syncthreads();  // previous chunk's dQ reads of ds_s / xch are done
    cstamp(c0, 2);
#pragma unroll
    for (int i = 0; i < 16; ++i) ds_s[acc_row(i, h) * DS_ROW + mykey + r] = from_f<bf16>(dp[i]);  // 0: idle wave
    __syncthreads();
    cstamp(c0, 3);
    if constexpr (DQ2) {
      // waves W0, W0 + 1 (SIMDs that do not host the 9-wave form's ninth wave): d tile wave - W0
      constexpr int W0 = NW == 9 ? 1 : 0;
      if (wave == W0 || wave == W0 + 1) {
        const int dtq = wave - W0;
        f32x16 acc = (f32x16){};
        if constexpr (DQ2 == 1) {
          // software-pipelined: the operand reads of k-steps st + 2, st + 3 are issued before the
          // MFMAs of st, st + 1 (left to itself the compiler sinks each pair of reads to its MFMAs and
          // waits on them: A1 backward 38.5 -> 37.7 us, A3 32.9 -> 32.6, bitwise the same)
          constexpr int NS = 2 * NW;
          const bf16* da = ds_s + r * DS_ROW + 8 * h;
          const bf16* kb = kt_s + (dtq * 32 + r) * KT_ROW + 8 * h;
          bf16x8 fa[4], fb[4];
#pragma unroll
          for (int st = 0; st < 2; ++st) { fa[st] = load8(da + st * 16); fb[st] = load8(kb + st * 16); }
#pragma unroll
          for (int st = 0; st < NS; st += 2) {
#pragma unroll
            for (int u = 2; u < 4; ++u)
              if (st + u < NS) { fa[(st + u) & 3] = load8(da + (st + u) * 16); fb[(st + u) & 3] = load8(kb + (st + u) * 16); }
            __builtin_amdgcn_sched_barrier(0);
            mma16(acc, fa[st & 3], fb[st & 3]);
            if (st + 1 < NS) mma16(acc, fa[(st + 1) & 3], fb[(st + 1) & 3]);
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {   // DQ2 == 2 (diagnostic build): the reads just in time
#pragma unroll
        for (int st = 0; st < 2 * NW; ++st) {
          const int kk = st * 16 + 8 * h;
          mma16(acc, load8(ds_s + r * DS_ROW + kk), load8(kt_s + (dtq * 32 + r) * KT_ROW + kk));
        }
        }
        cstamp(c0, 4);
        if (MODE == MODE_A1 && a.dqkv) {
          const int bag = bh / nh, hh = bh % nh, ld = 3 * nh * DH;
          bf16* qo = (bf16*)a.dqkv + ((size_t)bag * a.q_total + q_begin + c0) * ld + hh * DH + dtq * 32 + r;
#pragma unroll
          for (int i = 0; i < 16; ++i) qo[(size_t)acc_row(i, h) * ld] = (bf16)(a.dq_scale * acc[i]);
        } else if (MODE == MODE_A3 && a.slab_bf16) {   // the fused A3 backward's dq~ partials as bf16
          bf16* dst = (bf16*)a.dq + (size_t)blk * a.slab_stride + bh * a.dq_bh + (size_t)(q_begin + c0) * DH + dtq * 32 + r;
#pragma unroll
          for (int i = 0; i < 16; ++i) dst[(size_t)acc_row(i, h) * DH] = (bf16)acc[i];
        } else {
          float* dst = MODE == MODE_A1 ? a.dq + bh * a.dq_bh : a.dq + (size_t)blk * a.slab_stride + bh * a.dq_bh;
          dst += (size_t)(q_begin + c0) * DH + dtq * 32 + r;
#pragma unroll
          for (int i = 0; i < 16; ++i) dst[(size_t)acc_row(i, h) * DH] = acc[i];
        }
        cstamp(c0, 5);
      }
    } else {
    // dQ chunk [32 q x 64 d] = dS [32 x NK] . K [NK x 64]: this wave: d tile dt_q, keys 16 KQS kq ..
      f32x16 acc = (f32x16){};
      float* dst = MODE == MODE_A1 ? a.dq + bh * a.dq_bh : a.dq + (size_t)blk * a.slab_stride + bh * a.dq_bh;
      dst += (size_t)(q_begin + c0) * DH;
      if (dq_role) {
#pragma unroll
        for (int st = 0; st < KQS; ++st) {
          const int kk = kq * 16 * KQS + st * 16 + 8 * h;
          mma16(acc, load8(ds_s + r * DS_ROW + kk), load8(kt_s + (dt_q * 32 + r) * KT_ROW + kk));
        }
        // [32 q][64 d] partials of key group kq (9 waves: every group, 3 x 8 KB; 8 waves: groups 1-3)
        if (NW == 9 || kq > 0) {
          float* xs = xch + (NW == 9 ? kq : kq - 1) * 2048;
#pragma unroll
          for (int i = 0; i < 16; ++i) xs[acc_row(i, h) * 64 + dt_q * 32 + r] = acc[i];
        }
      }
      cstamp(c0, 4);
      __syncthreads();
      cstamp(c0, 5);
      if constexpr (NW == 9) {
        // every thread: one 4-column piece of the chunk's dq, the key groups summed in a fixed order
        if (tid < 512) {
          const int q = tid >> 4, d4 = (tid & 15) * 4;
          const f32x4 v = (*(const f32x4*)(xch + q * 64 + d4) + *(const f32x4*)(xch + 2048 + q * 64 + d4)) +
                          *(const f32x4*)(xch + 4096 + q * 64 + d4);
          if (MODE == MODE_A3 && a.slab_bf16)
            *(bf16x4*)((bf16*)a.dq + (size_t)blk * a.slab_stride + bh * a.dq_bh + (size_t)(q_begin + c0 + q) * DH + d4) =
                (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          else
            *(f32x4*)(dst + (size_t)q * DH + d4) = v;
        }
      } else if (kq == 0) {
        if (MODE == MODE_A1 && a.dqkv) {
          // bf16 q rows of dqkv (half the bytes of the fp32 rows; the landmark term is added in place
          // by tm_nys_assemble_q_slab_inplace)
          const int bag = bh / nh, hh = bh % nh, ld = 3 * nh * DH;
          bf16* qo = (bf16*)a.dqkv + ((size_t)bag * a.q_total + q_begin + c0) * ld + hh * DH + dt_q * 32 + r;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float v = acc[i];
#pragma unroll
            for (int g = 0; g < NKQ - 1; ++g) v += xch[g * 2048 + acc_row(i, h) * 64 + dt_q * 32 + r];
            qo[(size_t)acc_row(i, h) * ld] = (bf16)(a.dq_scale * v);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float v = acc[i];
#pragma unroll
            for (int g = 0; g < NKQ - 1; ++g) v += xch[g * 2048 + acc_row(i, h) * 64 + dt_q * 32 + r];
            dst[(size_t)acc_row(i, h) * DH + dt_q * 32 + r] = v;
          }
        }
      }
      cstamp(c0, 6);
    }
    if (c0 == 0) stamp(3);
    if (c0 == 96) stamp(4);
  }
  stamp(5);
  // ---- key-side epilogue through LDS (transpose to [key][d]) ----
  __syncthreads();
  if (MODE == MODE_A3 && a.dqkv) {
    // fused: the final bf16 k / v rows of dqkv (no fp32 key-side slabs, no assemble pass for them):
    // the conv backward's dv window loads issued first, dV and dK staged side by side, the dk~ / l
    // loads, one barrier, then 16-B bf16 stores of 8 columns per item
    constexpr int IT = (LY::NK * DH / 8 + NT - 1) / NT;
    static_assert(2 * LY::NK * 68 * 4 <= LY::BYTES, "fused A3 epilogue: two staged tiles exceed the layout");
    const int bag = bh / nh, hh = bh % nh, inner = nh * DH;
    bf16* outk = (bf16*)a.dqkv + ((size_t)bag * a.n_key_rows + key0) * 3 * inner + inner + hh * DH;
    bf16* outv = outk + inner;
    const bf16* dvc = (const bf16*)a.dv + bh * a.dv_bh + (size_t)key0 * DH;   // the conv backward's dv (bf16)
    const float* dkl = a.dkl + (size_t)bh * NL * DH;
    f32x4 av[IT][2], ak[IT][2];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + NT * it, key = i >> 3, d8 = (i & 7) * 8;
      const bool valid = key < nk;
      const bool vw = valid && key0 + key >= a.dv_lo && key0 + key < a.dv_hi;
      const bf16x8 pv = vw ? *(const bf16x8*)(dvc + (size_t)min(key, nk - 1) * DH + d8) : (bf16x8){};
      av[it][0] = (f32x4){(float)pv[0], (float)pv[1], (float)pv[2], (float)pv[3]};
      av[it][1] = (f32x4){(float)pv[4], (float)pv[5], (float)pv[6], (float)pv[7]};
    }
    float* stage_k = stage + LY::NK * 68;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int o = (mykey + r) * 68 + dt * 32 + 8 * g4 + 4 * h;
        *(f32x4*)(stage + o) = (f32x4){dvt[dt][4 * g4], dvt[dt][4 * g4 + 1], dvt[dt][4 * g4 + 2], dvt[dt][4 * g4 + 3]};
        *(f32x4*)(stage_k + o) = (f32x4){dkt[dt][4 * g4], dkt[dt][4 * g4 + 1], dkt[dt][4 * g4 + 2], dkt[dt][4 * g4 + 3]};
      }
    // dk~ / l rows (L2-resident: 256 x 64 per head) once dV / dK have left the registers
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + NT * it, key = min(i >> 3, nk - 1), d8 = (i & 7) * 8;
      const float* pk = dkl + (size_t)((key0 + key) / a.l) * DH + d8;
      ak[it][0] = *(const f32x4*)pk;
      ak[it][1] = *(const f32x4*)(pk + 4);
    }
    __syncthreads();
    const float il = a.inv_l;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + NT * it, key = i >> 3, d8 = (i & 7) * 8;
      if (key >= nk) continue;
      const float* sv = stage + key * 68 + d8;
      const float* sk = stage_k + key * 68 + d8;
      const f32x4 v0 = *(const f32x4*)sv + av[it][0], v1 = *(const f32x4*)(sv + 4) + av[it][1];
      const f32x4 k0 = *(const f32x4*)sk + ak[it][0] * il, k1 = *(const f32x4*)(sk + 4) + ak[it][1] * il;
      *(bf16x8*)(outv + (size_t)key * 3 * inner + d8) =
          (bf16x8){(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3], (bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
      *(bf16x8*)(outk + (size_t)key * 3 * inner + d8) =
          (bf16x8){(bf16)k0[0], (bf16)k0[1], (bf16)k0[2], (bf16)k0[3], (bf16)k1[0], (bf16)k1[1], (bf16)k1[2], (bf16)k1[3]};
    }
    stamp(6);
    return;
  }
#pragma unroll
  for (int which = 0; which < 2; ++which) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const f32x16& accv = which == 0 ? dvt[dt] : dkt[dt];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *(f32x4*)(stage + (mykey + r) * 68 + dt * 32 + 8 * g4 + 4 * h) =
            (f32x4){accv[4 * g4], accv[4 * g4 + 1], accv[4 * g4 + 2], accv[4 * g4 + 3]};
    }
    __syncthreads();
    if (MODE == MODE_A1 && a.slab_bf16) {
      bf16* dstb = (bf16*)(which == 0 ? a.dv : a.dk) + (size_t)blk * a.slab_stride + bh * (which == 0 ? a.dv_bh : a.dk_bh);
      for (int i = tid; i < nk * DH / 4; i += NT) {
        const int key = i >> 4, d4 = (i & 15) * 4;
        const f32x4 val = *(const f32x4*)(stage + key * 68 + d4);
        *(bf16x4*)(dstb + (size_t)key * DH + d4) = (bf16x4){(bf16)val[0], (bf16)val[1], (bf16)val[2], (bf16)val[3]};
      }
      __syncthreads();
      continue;
    }
    float* dst;
    bool add = false;
    if (MODE == MODE_A3) {
      dst = (which == 0 ? a.dv + bh * a.dv_bh : a.dk + bh * a.dk_bh) + (size_t)key0 * DH;
      add = (which == 0);
    } else {
      dst = (which == 0 ? a.dv : a.dk) + (size_t)blk * a.slab_stride + bh * (which == 0 ? a.dv_bh : a.dk_bh);
    }
    for (int i = tid; i < nk * DH / 4; i += NT) {
      const int key = i >> 4, d4 = (i & 15) * 4;
      f32x4 val = *(const f32x4*)(stage + key * 68 + d4);
      float* p = dst + (size_t)key * DH + d4;
      if (add) val += *(const f32x4*)p;
      *(f32x4*)p = val;
    }
    __syncthreads();
  }
  stamp(6);
}

template <typename T>
constexpr size_t bwd_smem_bytes() {
  return BwdLay<T>::BYTES;
}

// ---------------------------------------------------------------------------
// dqkv[bag][t][which*h*64 + head*64 + d]:
//   q: scale * (dq[t] + dql[t/l] / l);  k: dk[t] + dkl[t/l] / l;  v: dv[t]
template <typename T>
__global__ void assemble_dqkv_kernel(const float* __restrict__ dq, const float* __restrict__ dql,
                                     const float* __restrict__ dk, const float* __restrict__ dkl,
                                     const float* __restrict__ dv, int n, int l, int nh, float scale,
                                     T* __restrict__ dqkv) {
  // item = (t, 8 consecutive columns of the 3*nh*64-wide row) of bag blockIdx.y;
  // grid (ceil(n * 3*nh*8 / 256), nbags), block 256.
  const int inner = nh * DH, per_row = 3 * inner / 8;
  const long long item = (long long)blockIdx.x * 256 + threadIdx.x;
  if (item >= (long long)n * per_row) return;
  const int c = (int)(item % per_row) * 8;
  const int t = (int)(item / per_row), bag = blockIdx.y;
  const int which = c / inner, head = (c % inner) / DH, d = c % DH;
  const size_t bh = (size_t)bag * nh + head;
  const size_t row = (bh * n + t) * DH + d;
  const size_t lrow = (bh * NL + t / l) * DH + d;
  const float inv_l = 1.0f / (float)l;
  const float* src = which == 0 ? dq : which == 1 ? dk : dv;
  const float* lsrc = which == 0 ? dql : dkl;
  const f32x4 a0 = *(const f32x4*)(src + row), a1 = *(const f32x4*)(src + row + 4);
  f32x4 b0 = (f32x4){}, b1 = (f32x4){};
  if (which < 2) { b0 = *(const f32x4*)(lsrc + lrow); b1 = *(const f32x4*)(lsrc + lrow + 4); }
  const float a[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
  const float b[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  vec8<T> out;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float val;
    if (which == 0) val = scale * (a[e] + b[e] * inv_l);
    else if (which == 1) val = a[e] + b[e] * inv_l;
    else val = a[e];
    out[e] = from_f<T>(val);
  }
  store8<T>(dqkv + ((size_t)bag * n + t) * (3 * inner) + c, out);
}

// q part of dqkv only (the k / v parts written by the fused A3 backward):
// q = scale * (dq + (dql_a + dql_b)[t / l] / l); grid (ceil(n * nh * 8 / 256), nbags), block 256
template <typename T>
__global__ void assemble_q_kernel(const float* __restrict__ dq, int dq_row, const float* __restrict__ dql_a,
                                  const float* __restrict__ dql_b, int n, int l, int nh, float scale,
                                  T* __restrict__ dqkv) {
  const int inner = nh * DH, per_row = inner / 8;
  const long long item = (long long)blockIdx.x * 256 + threadIdx.x;
  if (item >= (long long)n * per_row) return;
  const int c = (int)(item % per_row) * 8;
  const int t = (int)(item / per_row), bag = blockIdx.y;
  const int head = c / DH, d = c % DH;
  const size_t bh = (size_t)bag * nh + head;
  const size_t row = (bh * n + t) * DH + d;
  const size_t lrow = (bh * NL + t / l) * DH + d;
  const float inv_l = 1.0f / (float)l;
  const f32x8 a = (dq_row < 0 || t == dq_row) ? load8<float>(dq + row) : (f32x8){};  // dq_row: the only non-zero row
  const f32x8 b0 = load8<float>(dql_a + lrow), b1 = load8<float>(dql_b + lrow);
  vec8<T> out;
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] = from_f<T>(scale * (a[e] + (b0[e] + b1[e]) * inv_l));
  store8<T>(dqkv + ((size_t)bag * n + t) * (3 * inner) + c, out);
}

// q part of dqkv with the A3 backward's dq~ partial slab reduced in the same launch (no separate
// split-K reduce, no dq~3 round trip): q = scale * (dq + (dql + sum_p slab[p])[t / l] / l).
// grid (256 landmarks, nbags), block 512: the workgroup's first QP dq pieces per thread are
// requested first, then landmark j's slab row is summed (eight part groups, combined in a fixed
// order) while they are in flight, then the l tokens of segment j are written.
// INPLACE (bf16): the q rows already hold bf16(scale * dq) (tm_nys_a1_bwd_dqkv); the landmark term
// scale * (dql + sum_p slab[p])[t / l] / l is added to them in place.
constexpr int AQ_THREADS = 512, AQ_GROUPS = AQ_THREADS / 64, AQ_QP = 5;
template <typename T, bool INPLACE = false>
__global__ __launch_bounds__(AQ_THREADS) void assemble_q_slab_kernel(const float* __restrict__ dq, int dq_row,
                                                                     const float* __restrict__ dql,
                                                                     const bf16* __restrict__ slab, int slabs,
                                                                     long long slab_count, int n, int l, int nh,
                                                                     float scale, T* __restrict__ dqkv) {
  __shared__ __attribute__((aligned(16))) float part[AQ_GROUPS][8 * DH];   // [group][nh <= 8 heads x 64 d]
  const int j = blockIdx.x, bag = blockIdx.y, tid = threadIdx.x;
  const int inner = nh * DH, pieces = inner / 8;                          // <= 64
  const int items = l * pieces;
  auto dq_row_of = [&](int it, int& t, int& c) -> size_t {
    t = j * l + it / pieces;
    c = (it % pieces) * 8;
    return (((size_t)bag * nh + c / DH) * n + t) * DH + c % DH;
  };
  auto load_q = [&](int it) -> f32x8 {
    int t, c;
    const size_t row = dq_row_of(it, t, c);
    if constexpr (INPLACE) {
      const vec8<T> v = load8<T>(dqkv + ((size_t)bag * n + t) * (3 * inner) + c);
      f32x8 r;
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = to_f(v[e]);
      return r;
    } else {
      return (dq_row < 0 || t == dq_row) ? load8<float>(dq + row) : (f32x8){};
    }
  };
  f32x8 a[AQ_QP];
#pragma unroll
  for (int u = 0; u < AQ_QP; ++u) {
    const int it = tid + AQ_THREADS * u;
    a[u] = it < items ? load_q(it) : (f32x8){};
  }
  {
    const int pc = tid & 63, g = tid >> 6;
    if (pc < pieces) {
      const int c = pc * 8, head = c / DH, d = c % DH;
      const size_t off = (((size_t)bag * nh + head) * NL + j) * DH + d;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int p = g;
      for (; p + 3 * AQ_GROUPS < slabs; p += 4 * AQ_GROUPS) {   // four partials in flight per thread
        bf16x8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = load8<bf16>(slab + (size_t)(p + AQ_GROUPS * u) * slab_count + off);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += (float)v[u][e];
      }
      for (; p < slabs; p += AQ_GROUPS) {
        const bf16x8 v = load8<bf16>(slab + (size_t)p * slab_count + off);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) part[g][c + e] = acc[e];
    }
  }
  __syncthreads();
  for (int col = tid; col < inner; col += AQ_THREADS) {   // pairwise over the groups, then the landmark path's dq~
    const int head = col / DH, d = col % DH;
    const float sum = ((part[0][col] + part[1][col]) + (part[2][col] + part[3][col])) +
                      ((part[4][col] + part[5][col]) + (part[6][col] + part[7][col]));
    part[0][col] = (dql[(((size_t)bag * nh + head) * NL + j) * DH + d] + sum) * (1.0f / (float)l);
  }
  __syncthreads();
  auto store = [&](int it, const f32x8& av) {
    int t, c;
    (void)dq_row_of(it, t, c);
    vec8<T> out;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      out[e] = INPLACE ? from_f<T>(av[e] + scale * part[0][c + e]) : from_f<T>(scale * (av[e] + part[0][c + e]));
    store8<T>(dqkv + ((size_t)bag * n + t) * (3 * inner) + c, out);
  };
#pragma unroll
  for (int u = 0; u < AQ_QP; ++u)
    if (tid + AQ_THREADS * u < items) store(tid + AQ_THREADS * u, a[u]);
  for (int it = tid + AQ_THREADS * AQ_QP; it < items; it += AQ_THREADS)   // long segments (l > 40)
    store(it, load_q(it));
}

}  // namespace

// ============================ C entry points ===============================
#ifdef TM_DIAG
extern "C" void tm_debug_set_nys_variant(int value) { g_nys_variant = value; }
// copy the VAR 9 a1_fwd stamps ([block][wave][8] u64) to a host buffer (diagnostics only)
extern "C" int tm_debug_a1_stamps(unsigned long long* host, int count) {
  TM_REQUIRE(count > 0 && count <= 512 * 8 * 8, "a1_stamps: bad count");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_a1_stamps), count * sizeof(unsigned long long)) != hipSuccess) {
    tm_set_error("a1_stamps: copy");
    return 2;
  }
  return 0;
}
#endif

#define TM_DTYPE_DISPATCH(dt, CALL)                               \
  if ((dt) == TM_BF16) { using T = bf16; CALL; }                  \
  else if ((dt) == TM_F32) { using T = float; CALL; }             \
  else { tm_set_error("nystrom: dtype must be TM_F32 or TM_BF16"); return 1; }

extern "C" int tm_nys_landmarks(int dtype, const void* q, const void* k, int nbh, int n, float* ql, float* kl,
                                void* ql_t, void* kl_t, void* stream) {
  TM_REQUIRE(n > 0 && n % NL == 0, "landmarks: n must be a positive multiple of 256");
  const int l = n / NL;
  TM_DTYPE_DISPATCH(dtype, (landmarks_kernel<T><<<dim3(nbh, NL / 8), 256, 0, (hipStream_t)stream>>>(
                               (const T*)q, (const T*)k, n, l, ql, kl, (T*)ql_t, (T*)kl_t)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_sim2_softmax(const float* ql, const float* kl, int nbh, float* a2, void* stream) {
  sim2_softmax_kernel<<<dim3(nbh, NL / S2_ROWS), 256, 0, (hipStream_t)stream>>>(ql, kl, a2, nullptr);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_sim2_softmax_split(const float* ql, const float* kl, int nbh, float* a2, void* a2s,
                                         void* stream) {
  TM_REQUIRE(a2s, "sim2_softmax_split: a2s is required");
#ifdef TM_DIAG
  if (NYS_VARIANT == 21)   // the MFMA form (measured slower: 15.1 vs 12 us with 64 workgroups)
    sim2_softmax_mfma_kernel<<<dim3(nbh, NL / 32), 512, 0, (hipStream_t)stream>>>(ql, kl, a2, (bf16*)a2s);
  else
#endif
    sim2_softmax_kernel<<<dim3(nbh, NL / S2_ROWS), 256, 0, (hipStream_t)stream>>>(ql, kl, a2, (bf16*)a2s);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_softmax_bwd_rows256(const float* a, const float* da, float* ds, int rows, void* stream) {
  softmax_bwd_rows_kernel<<<(rows + 3) / 4, 256, 0, (hipStream_t)stream>>>(a, da, ds, rows);
  TM_CHECK_LAUNCH();
  return 0;
}

// key splits (partials per head) of the bf16 A3 forward
extern "C" long long tm_nys_a3_partials(int nbh, int n) { return a3v_splits(nbh, n); }

extern "C" long long tm_nys_a3_workspace(int nbh, int n) {
  const long long parts = std::max((long long)(n / NL), (long long)a3v_splits(nbh, n));
  return parts * nbh * NL * (DH + 2) * (long long)sizeof(float);
}

namespace {
// the bf16 key-split launch (+ the fused A2 rows when s2.a2 is set and the split allows it)
void launch_a3_fwd_v2(const float* ql, const void* k, const void* v, int nbh, int n, float* work, Sim2Out s2,
                      hipStream_t st) {
  const int P = a3v_splits(nbh, n);
  bf16* po = (bf16*)work;                          // bf16 partial sums in the first half of an fp32-sized region
  float* pm = work + (size_t)P * nbh * NL * DH;
  float* pl = pm + (size_t)P * nbh * NL;
  const dim3 grid(P, nbh);
  const bf16* kb = (const bf16*)k;
  const bf16* vb = (const bf16*)v;
#ifdef TM_DIAG
  if (NYS_VARIANT == 32 && !s2.a2) {   // diagnostic: s_memtime stamps per wave (tm_debug_a1_stamps)
    tm_allow_smem(a3_fwd_v2_kernel<1>, A3V_BYTES);
    a3_fwd_v2_kernel<1><<<grid, 512, A3V_BYTES, st>>>(ql, kb, vb, n, P, po, pm, pl, s2);
    return;
  }
  if (NYS_VARIANT == 32 && s2.a2 && P * 8 == NL) {   // the same with the fused A2 rows
    tm_allow_smem(a3_fwd_v2_kernel<1, 4>, A3V_BYTES);
    a3_fwd_v2_kernel<1, 4><<<grid, 512, A3V_BYTES, st>>>(ql, kb, vb, n, P, po, pm, pl, s2);
    return;
  }
#endif
  if (s2.a2 && P * 8 == NL) {
    tm_allow_smem(a3_fwd_v2_kernel<0, 4>, A3V_BYTES);
    a3_fwd_v2_kernel<0, 4><<<grid, 512, A3V_BYTES, st>>>(ql, kb, vb, n, P, po, pm, pl, s2);
  } else if (s2.a2 && P * 16 == NL) {
    tm_allow_smem(a3_fwd_v2_kernel<0, 8>, A3V_BYTES);
    a3_fwd_v2_kernel<0, 8><<<grid, 512, A3V_BYTES, st>>>(ql, kb, vb, n, P, po, pm, pl, s2);
  } else {
    tm_allow_smem(a3_fwd_v2_kernel<0>, A3V_BYTES);
    a3_fwd_v2_kernel<0><<<grid, 512, A3V_BYTES, st>>>(ql, kb, vb, n, P, po, pm, pl, s2);
    if (s2.a2)   // a split the fused rows do not tile: the separate launch
      sim2_softmax_kernel<<<dim3(nbh, NL / S2_ROWS), 256, 0, st>>>(ql, s2.kl, s2.a2, s2.a2s);
  }
}
}  // namespace

extern "C" int tm_nys_a3_fwd(int dtype, const float* ql, const void* k, const void* v, int nbh, int n, float* work,
                             float* w, float* lse3, void* stream) {
  TM_REQUIRE(n > 0 && n % NL == 0, "a3_fwd: n must be a positive multiple of 256");
  TM_REQUIRE((w && lse3) || dtype == TM_BF16, "a3_fwd: w / lse3 may be null (deferred combine) in bf16 mode only");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16) {
    launch_a3_fwd_v2(ql, k, v, nbh, n, work, Sim2Out{nullptr, nullptr, nullptr}, st);
    TM_CHECK_LAUNCH();
    if (!w) return 0;   // deferred: the combine runs in the pseudo-inverse chain (tm_pinv_fwd_split_a3)
    const int P = a3v_splits(nbh, n);
    const bf16* po = (const bf16*)work;
    float* pm = work + (size_t)P * nbh * NL * DH;
    float* pl = pm + (size_t)P * nbh * NL;
    a3_combine_v2_kernel<<<dim3(nbh, NL / 8), 256, 0, st>>>(A3Combine{po, pm, pl, P, nbh, w, lse3});
    TM_CHECK_LAUNCH();
    return 0;
  }
  const int nkb = n / NL;
  float* po = work;
  float* pm = po + (size_t)nkb * nbh * NL * DH;
  float* pl = pm + (size_t)nkb * nbh * NL;
  TM_DTYPE_DISPATCH(dtype, ({
    const size_t sm = ((size_t)NL * Lay<T>::KROW + Lay<T>::VELEMS) * sizeof(T);
    tm_allow_smem(a3_fwd_kernel<T>, sm);
    a3_fwd_kernel<T><<<dim3(nkb, nbh, 2), 256, sm, st>>>(ql, (const T*)k, (const T*)v, n, po, pm, pl);
  }));
  TM_CHECK_LAUNCH();
  a3_combine_kernel<<<dim3(nbh, NL / 16), 256, 0, st>>>(po, pm, pl, nkb, nbh, w, lse3);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_a3_fwd_sim2(const float* ql, const float* kl, const void* k, const void* v, int nbh, int n,
                                  float* work, float* a2, void* a2s, void* stream) {
  TM_REQUIRE(n > 0 && n % NL == 0, "a3_fwd_sim2: n must be a positive multiple of 256");
  TM_REQUIRE(ql && kl && k && v && work && a2 && a2s, "a3_fwd_sim2: null operand");
  launch_a3_fwd_v2(ql, k, v, nbh, n, work, Sim2Out{kl, a2, (bf16*)a2s}, (hipStream_t)stream);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_a1_fwd(int dtype, const void* q, const void* v, const void* kl_t, const void* y_t,
                             const float* wconv, int nbh, int nh, int n, void* merged, float* lse1, void* stream) {
  TM_REQUIRE(n > 0 && n % NL == 0 && nbh % nh == 0, "a1_fwd: bad shape");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16 && NYS_VARIANT != 14) {
    const int cph = n / 32;
    int wpg = std::max(1, std::min(tm_cu_count() / std::max(nbh, 1), cph));
    wpg = std::max(wpg, (cph + A1P_MAXCH - 1) / A1P_MAXCH);  // <= A1P_MAXCH chunks per workgroup
#ifdef TM_DIAG
    // ablation variants 11-19 (microbench only): 10 + VAR
    auto kern = NYS_VARIANT == 11 ? a1_fwd_bf16_kernel<1> : NYS_VARIANT == 12 ? a1_fwd_bf16_kernel<2>
              : NYS_VARIANT == 13 ? a1_fwd_bf16_kernel<3> : NYS_VARIANT == 19 ? a1_fwd_bf16_kernel<9>
              : NYS_VARIANT == 16 ? a1_fwd_bf16_kernel<6> : a1_fwd_bf16_kernel<0>;
#else
    auto kern = a1_fwd_bf16_kernel<0>;
#endif
    tm_allow_smem(kern, A1P_BYTES);
    kern<<<dim3(wpg, nbh), 256, A1P_BYTES, st>>>((const bf16*)q, (const bf16*)v, (const bf16*)kl_t,
                                                               (const bf16*)y_t, wconv, n, nh, wpg, (bf16*)merged,
                                                               lse1);
    TM_CHECK_LAUNCH();
    return 0;
  }
  TM_DTYPE_DISPATCH(dtype, ({
    const size_t sm1 = ((size_t)NL * Lay<T>::KROW + Lay<T>::VELEMS) * sizeof(T);
    const size_t sm = sm1 > A1_EPI_BYTES ? sm1 : A1_EPI_BYTES;
#ifdef TM_DIAG
    auto kern = NYS_VARIANT == 1 ? a1_fwd_kernel<T, 1> : NYS_VARIANT == 2 ? a1_fwd_kernel<T, 2> : a1_fwd_kernel<T, 0>;
#else
    auto kern = a1_fwd_kernel<T, 0>;
#endif
    tm_allow_smem(kern, sm);
    kern<<<dim3(n / 128, nbh), 256, sm, st>>>((const T*)q, (const T*)v, (const T*)kl_t,
                                              (const T*)y_t, wconv, n, nh, (T*)merged, lse1);
  }));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_rowdot_cast(int dtype, const float* dw, const float* w, int rows, float* dd, void* dw_t,
                                  void* stream) {
  TM_DTYPE_DISPATCH(dtype, (rowdot_cast_kernel<T><<<(rows + 3) / 4, 256, 0, (hipStream_t)stream>>>(
                               dw, w, dd, (T*)dw_t, rows)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_cast_f32(int dtype, const float* x, void* y, long long count, void* stream) {
  if (count == 0) return 0;
  TM_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0, "cast_f32: 16-B aligned buffers");
  TM_DTYPE_DISPATCH(dtype, (cast_rows_kernel<T><<<(unsigned)((count + 2047) / 2048), 256, 0, (hipStream_t)stream>>>(
                               x, (T*)y, count)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_nys_conv_bwd_workspace(int nbags, int nh, int n) {
  const int r = conv_bwd_rows(nbags * nh, n);
  const long long blocks = std::max((n + 63) / 64, (n + r - 1) / r);
  return (long long)nbags * blocks * nh * TAPS * (long long)sizeof(float);
}

extern "C" int tm_nys_conv_bwd(int dtype, const void* dmerged, const void* merged, const void* v, const float* wconv,
                               int nbh, int nh, int n, void* dv, float* d1, float* work, float* dwconv,
                               tm_reduce_queue* rq, void* stream) {
  TM_REQUIRE(nbh % nh == 0 && n > 0, "conv_bwd: bad shape");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16 && NYS_VARIANT != 7) {
    const int r = conv_bwd_rows(nbh, n), nblk = (n + r - 1) / r;
    tm_allow_smem(conv_bwd_mfma_kernel, CbLay::BYTES);
    conv_bwd_mfma_kernel<<<dim3(nblk, nbh), 512, CbLay::BYTES, st>>>(
        (const bf16*)dmerged, (const bf16*)merged, (const bf16*)v, wconv, n, nh, r, (bf16*)dv, d1, work);
    TM_CHECK_LAUNCH();
    return tm_splitk_reduce(work, dwconv, (nbh / nh) * nblk, (long long)nh * TAPS, 1.0f, 0, rq, stream);
  }
  const int ntb = (n + 63) / 64;
  TM_DTYPE_DISPATCH(dtype, (conv_bwd_kernel<T><<<dim3(ntb, nbh), 256, 0, st>>>(
                               (const T*)dmerged, (const T*)merged, (const T*)v, wconv, n, nh, (T*)dv, d1, work)));
  TM_CHECK_LAUNCH();
  return tm_splitk_reduce(work, dwconv, (nbh / nh) * ntb, (long long)nh * TAPS, 1.0f, 0, rq, stream);
}

// A1 backward: keys = landmarks kl_t [bh][256][64], values = y_t, queries = q rows, dO = dmerged.
// dq (fp32 [bh][n][64]) written; dkl/dy partial slabs [n/qpw][bh][256][64] in work.
namespace {
// workgroups per head of the bf16 A1 backward (even split of the n / 32 query chunks)
int a1_bwd_split(int nbh, int n) {
  const int cph = n / 32;
  const int w = std::min(cph, std::max(1, tm_cu_count() / std::max(nbh, 1)));
  return std::max(w, (cph + BwdLay16::MAXQ / 32 - 1) / (BwdLay16::MAXQ / 32));
}
}  // namespace

extern "C" long long tm_nys_a1_bwd_workspace(int nbh, int n, int queries_per_wg) {
  const long long slabs = std::max((long long)(n / queries_per_wg), (long long)a1_bwd_split(nbh, n));
  return 2LL * slabs * nbh * NL * DH * (long long)sizeof(float);
}

namespace {
int a1_bwd_impl(int dtype, const void* q, const void* dmerged, const void* kl_t, const void* y_t, const float* lse1,
                const float* d1, int nbh, int nh, int n, int queries_per_wg, float* dq, void* dqkv, float dq_scale,
                float* work, float* dkl, float* dy, int accumulate, tm_reduce_queue* rq, void* stream);
}  // namespace

extern "C" int tm_nys_a1_bwd(int dtype, const void* q, const void* dmerged, const void* kl_t, const void* y_t,
                             const float* lse1, const float* d1, int nbh, int nh, int n, int queries_per_wg,
                             float* dq, float* work, float* dkl, float* dy, int accumulate, tm_reduce_queue* rq,
                             void* stream) {
  return a1_bwd_impl(dtype, q, dmerged, kl_t, y_t, lse1, d1, nbh, nh, n, queries_per_wg, dq, nullptr, 0.f, work, dkl,
                     dy, accumulate, rq, stream);
}

// bf16 only: dq goes to the q part of dqkv as bf16(dq_scale * dq) (tm_nys_assemble_q_slab_inplace
// then adds the landmark term in place)
extern "C" int tm_nys_a1_bwd_dqkv(const void* q, const void* dmerged, const void* kl_t, const void* y_t,
                                  const float* lse1, const float* d1, int nbh, int nh, int n, void* dqkv,
                                  float dq_scale, float* work, float* dkl, float* dy, tm_reduce_queue* rq,
                                  void* stream) {
  TM_REQUIRE(dqkv && ((uintptr_t)dqkv % 16) == 0 && nbh % nh == 0, "a1_bwd_dqkv: dqkv");
  return a1_bwd_impl(TM_BF16, q, dmerged, kl_t, y_t, lse1, d1, nbh, nh, n, 256, nullptr, dqkv, dq_scale, work, dkl,
                     dy, 0, rq, stream);
}

namespace {
int a1_bwd_impl(int dtype, const void* q, const void* dmerged, const void* kl_t, const void* y_t, const float* lse1,
                const float* d1, int nbh, int nh, int n, int queries_per_wg, float* dq, void* dqkv, float dq_scale,
                float* work, float* dkl, float* dy, int accumulate, tm_reduce_queue* rq, void* stream) {
  TM_REQUIRE(queries_per_wg % 32 == 0 && n % queries_per_wg == 0, "a1_bwd: queries_per_wg must divide n, x32");
  const bool split = dtype == TM_BF16 && queries_per_wg <= NL && NYS_VARIANT != 3;
  TM_REQUIRE(!dqkv || split, "a1_bwd_dqkv: the bf16 split kernel only");
  const int nqc = split ? a1_bwd_split(nbh, n) : n / queries_per_wg;
  BwdArgs a{};
  a.q = q; a.q_bag = (long long)nh * n * DH; a.q_head = (long long)n * DH; a.q_row = DH;
  a.dO = dmerged; a.o_bag = (long long)n * nh * DH; a.o_head = DH; a.o_row = nh * DH;
  a.k = kl_t; a.k_bag = (long long)nh * NL * DH; a.k_head = (long long)NL * DH;
  a.v = y_t; a.v_bag = a.k_bag; a.v_head = a.k_head;
  a.lse = lse1; a.lse_bh = n; a.dd = d1; a.dd_bh = n;
  a.dq = dq; a.dq_bh = (long long)n * DH;
  a.dqkv = dqkv; a.dq_scale = dq_scale;
  float* slab_k = work;
  float* slab_v = work + (size_t)nqc * nbh * NL * DH;
  a.dk = slab_k; a.dk_bh = (long long)NL * DH;
  a.dv = slab_v; a.dv_bh = (long long)NL * DH;
  a.slab_stride = (long long)nbh * NL * DH;
  a.nh = nh; a.n_queries_per_wg = queries_per_wg; a.n_key_rows = NL;
  hipStream_t st = (hipStream_t)stream;
  if (split) {
    a.q_total = n;
    // the dk~ / dY partials as bf16 (diagnostic variant 37: fp32, the earlier form)
    a.slab_bf16 = NYS_VARIANT != 37;
#ifdef TM_DIAG
    if (NYS_VARIANT == 33 || NYS_VARIANT == 34) {   // diagnostic: stamps per wave (33 phases, 34 inside chunk 2)
      auto kern = NYS_VARIANT == 33 ? attn_bwd_bf16_kernel<MODE_A1, 8, 1> : attn_bwd_bf16_kernel<MODE_A1, 8, 2>;
      tm_allow_smem(kern, BwdLay16::BYTES);
      kern<<<dim3(nqc, nbh), 512, BwdLay16::BYTES, st>>>(a);
    } else if (NYS_VARIANT == 35) {   // diagnostic: the earlier cross-wave dQ form
      tm_allow_smem(attn_bwd_bf16_kernel<MODE_A1, 8, 0, 0>, BwdLay16::BYTES);
      attn_bwd_bf16_kernel<MODE_A1, 8, 0, 0><<<dim3(nqc, nbh), 512, BwdLay16::BYTES, st>>>(a);
    } else if (NYS_VARIANT == 36) {   // diagnostic: the dQ chain with its reads just in time
      tm_allow_smem(attn_bwd_bf16_kernel<MODE_A1, 8, 0, 2>, BwdLay16::BYTES);
      attn_bwd_bf16_kernel<MODE_A1, 8, 0, 2><<<dim3(nqc, nbh), 512, BwdLay16::BYTES, st>>>(a);
    } else
#endif
    {
      tm_allow_smem(attn_bwd_bf16_kernel<MODE_A1>, BwdLay16::BYTES);
      attn_bwd_bf16_kernel<MODE_A1><<<dim3(nqc, nbh), 512, BwdLay16::BYTES, st>>>(a);
    }
  } else {
    TM_DTYPE_DISPATCH(dtype, (tm_allow_smem(attn_bwd_kernel<T, MODE_A1>, bwd_smem_bytes<T>()),
                              attn_bwd_kernel<T, MODE_A1><<<dim3(nqc, nbh), 512, bwd_smem_bytes<T>(), st>>>(a)));
  }
  TM_CHECK_LAUNCH();
  const long long cnt = (long long)nbh * NL * DH;
  const int sdt = a.slab_bf16 ? TM_BF16 : TM_F32;
  int rc = tm_splitk_reduce_typed(slab_k, sdt, dkl, nqc, cnt, 1.0f, accumulate, rq, stream);
  if (rc) return rc;
  return tm_splitk_reduce_typed(slab_v, sdt, dy, nqc, cnt, 1.0f, 0, rq, stream);
}
}  // namespace

// A3 backward: keys = k rows, values = v rows, queries = ql_t (256 landmarks), dO = dw_t.
// dk written (=), dv accumulated (+=), dql accumulated from partial slabs.
namespace {
// bf16 A3 backward grid: the head's n / 32 key units split evenly over 256 / nbh workgroups when
// that is <= 9 units each (one chip round; the 9-wave form), else over ceil(units / 8) workgroups
// of the 8-wave form.  Every workgroup writes one dq~ partial slab.
struct A3Split { int wpg, nw; };
A3Split a3_bwd_split(int nbh, int n) {
  const int units = n / 32;
  const int w = std::max(1, std::min(units, tm_cu_count() / std::max(nbh, 1)));
  const int per = (units + w - 1) / w;
  if (per <= 8) return {w, 8};
  if (per == 9) return {w, 9};
  return {(units + 7) / 8, 8};
}

void launch_a3_bwd_bf16(BwdArgs& a, int nbh, int n, hipStream_t st, int& slabs) {
  const A3Split sp = a3_bwd_split(nbh, n);
  a.q_total = n;  // even split on
  slabs = sp.wpg;
  if (sp.nw == 9) {
#ifdef TM_DIAG
    if (NYS_VARIANT == 30) {   // diagnostic: s_memtime stamps per wave (tm_debug_a1_stamps)
      tm_allow_smem(attn_bwd_bf16_kernel<MODE_A3, 9, 1>, BwdLay9::BYTES);
      attn_bwd_bf16_kernel<MODE_A3, 9, 1><<<dim3(sp.wpg, nbh), 576, BwdLay9::BYTES, st>>>(a);
      return;
    }
    if (NYS_VARIANT == 31) {   // diagnostic: stamps inside query chunk 2
      tm_allow_smem(attn_bwd_bf16_kernel<MODE_A3, 9, 2>, BwdLay9::BYTES);
      attn_bwd_bf16_kernel<MODE_A3, 9, 2><<<dim3(sp.wpg, nbh), 576, BwdLay9::BYTES, st>>>(a);
      return;
    }
    if (NYS_VARIANT == 35) {   // diagnostic: the earlier cross-wave dQ form
      tm_allow_smem(attn_bwd_bf16_kernel<MODE_A3, 9, 0, 0>, BwdLay9::BYTES);
      attn_bwd_bf16_kernel<MODE_A3, 9, 0, 0><<<dim3(sp.wpg, nbh), 576, BwdLay9::BYTES, st>>>(a);
      return;
    }
    if (NYS_VARIANT == 36) {   // diagnostic: the dQ chain with its reads just in time
      tm_allow_smem(attn_bwd_bf16_kernel<MODE_A3, 9, 0, 2>, BwdLay9::BYTES);
      attn_bwd_bf16_kernel<MODE_A3, 9, 0, 2><<<dim3(sp.wpg, nbh), 576, BwdLay9::BYTES, st>>>(a);
      return;
    }
#endif
    tm_allow_smem(attn_bwd_bf16_kernel<MODE_A3, 9>, BwdLay9::BYTES);
    attn_bwd_bf16_kernel<MODE_A3, 9><<<dim3(sp.wpg, nbh), 576, BwdLay9::BYTES, st>>>(a);
  } else {
    tm_allow_smem(attn_bwd_bf16_kernel<MODE_A3, 8>, BwdLay16::BYTES);
    attn_bwd_bf16_kernel<MODE_A3, 8><<<dim3(sp.wpg, nbh), 512, BwdLay16::BYTES, st>>>(a);
  }
}
}  // namespace

extern "C" long long tm_nys_a3_bwd_workspace(int nbh, int n) {
  const long long slabs = std::max((long long)(n / NL), (long long)a3_bwd_split(nbh, n).wpg);
  return slabs * nbh * NL * DH * (long long)sizeof(float);
}

extern "C" int tm_nys_a3_bwd(int dtype, const void* ql_t, const void* dw_t, const void* k, const void* v,
                             const float* lse3, const float* d3, int nbh, int nh, int n, float* dk, float* dv,
                             float* work, float* dql, int accumulate, tm_reduce_queue* rq, void* stream) {
  TM_REQUIRE(n % NL == 0, "a3_bwd: n must be a multiple of 256");
  const int nkb = n / NL;
  BwdArgs a{};
  a.q = ql_t; a.q_bag = (long long)nh * NL * DH; a.q_head = (long long)NL * DH; a.q_row = DH;
  a.dO = dw_t; a.o_bag = a.q_bag; a.o_head = a.q_head; a.o_row = DH;
  a.k = k; a.k_bag = (long long)nh * n * DH; a.k_head = (long long)n * DH;
  a.v = v; a.v_bag = a.k_bag; a.v_head = a.k_head;
  a.lse = lse3; a.lse_bh = NL; a.dd = d3; a.dd2 = d3 + (size_t)nbh * NL; a.dd_bh = NL;   // [2][nbh][256] partials
  a.dq = work; a.dq_bh = (long long)NL * DH;
  a.slab_stride = (long long)nbh * NL * DH;
  a.dk = dk; a.dk_bh = (long long)n * DH;
  a.dv = dv; a.dv_bh = (long long)n * DH;
  a.nh = nh; a.n_queries_per_wg = NL; a.n_key_rows = n;
  hipStream_t st = (hipStream_t)stream;
  int slabs = nkb;
  if (dtype == TM_BF16 && NYS_VARIANT != 3) {
    launch_a3_bwd_bf16(a, nbh, n, st, slabs);
  } else {
    TM_DTYPE_DISPATCH(dtype, (tm_allow_smem(attn_bwd_kernel<T, MODE_A3>, bwd_smem_bytes<T>()),
                              attn_bwd_kernel<T, MODE_A3><<<dim3(nkb, nbh), 512, bwd_smem_bytes<T>(), st>>>(a)));
  }
  TM_CHECK_LAUNCH();
  return tm_splitk_reduce(work, dql, slabs, (long long)nbh * NL * DH, 1.0f, accumulate, rq, stream);
}

// bf16 A3 backward with the fused key-side epilogue: the final k / v parts of dqkv from dK, dV,
// the conv backward's dv (fp32, read) and dk~ (fp32 [bh][256][64], after the pseudo-inverse
// backward); dql3 (=) from the per-key-block slabs.
extern "C" int tm_nys_a3_bwd_fused(const void* ql_t, const void* dw_t, const void* k, const void* v,
                                   const float* lse3, const float* d3, int nbh, int nh, int n, const void* dv_conv,
                                   int dv_lo, int dv_hi, const float* dkl, float* work, float* dql, void* dqkv,
                                   tm_reduce_queue* rq, void* stream) {
  TM_REQUIRE(n % NL == 0 && nbh % nh == 0, "a3_bwd_fused: n must be a multiple of 256");
  TM_REQUIRE(dv_conv && dkl && dqkv, "a3_bwd_fused: null operand");
  const int nkb = n / NL;
  BwdArgs a{};
  a.q = ql_t; a.q_bag = (long long)nh * NL * DH; a.q_head = (long long)NL * DH; a.q_row = DH;
  a.dO = dw_t; a.o_bag = a.q_bag; a.o_head = a.q_head; a.o_row = DH;
  a.k = k; a.k_bag = (long long)nh * n * DH; a.k_head = (long long)n * DH;
  a.v = v; a.v_bag = a.k_bag; a.v_head = a.k_head;
  a.lse = lse3; a.lse_bh = NL; a.dd = d3; a.dd2 = d3 + (size_t)nbh * NL; a.dd_bh = NL;   // [2][nbh][256] partials
  a.dq = work; a.dq_bh = (long long)NL * DH;
  a.slab_stride = (long long)nbh * NL * DH;
  a.dv = (float*)dv_conv; a.dv_bh = (long long)n * DH;   // bf16 rows (the kernel reads them as bf16)
  a.nh = nh; a.n_queries_per_wg = NL; a.n_key_rows = n;
  a.dqkv = dqkv; a.dkl = dkl; a.l = n / NL; a.inv_l = 1.0f / (float)(n / NL);
  a.dv_lo = dv_lo; a.dv_hi = dv_hi;
  hipStream_t st = (hipStream_t)stream;
  int slabs = nkb;
  a.slab_bf16 = 1;      // the dq~ partials as bf16 ([slabs][B*h][256][64], summed in fp32 by the consumer)
  launch_a3_bwd_bf16(a, nbh, n, st, slabs);
  TM_CHECK_LAUNCH();
  if (!dql) return 0;   // the slab stays for tm_nys_assemble_q_slab
  return tm_splitk_reduce_typed(work, TM_BF16, dql, slabs, (long long)nbh * NL * DH, 1.0f, 0, rq, stream);
}

extern "C" int tm_nys_a3_bwd_slabs(int nbh, int n) { return a3_bwd_split(nbh, n).wpg; }

extern "C" int tm_nys_assemble_q_slab(int dtype, const float* dq, int dq_row, const float* dql, const void* slab,
                                      int slabs, int nbags, int nh, int n, float scale, void* dqkv, void* stream) {
  TM_REQUIRE(n > 0 && n % NL == 0 && nh > 0 && nh <= 8 && slabs > 0, "assemble_q_slab: bad shape");
  TM_REQUIRE(dq && dql && slab && dqkv, "assemble_q_slab: null operand");
  TM_DTYPE_DISPATCH(dtype, (assemble_q_slab_kernel<T><<<dim3(NL, nbags), AQ_THREADS, 0, (hipStream_t)stream>>>(
                               dq, dq_row, dql, (const bf16*)slab, slabs, (long long)nbags * nh * NL * DH, n, n / NL,
                               nh, scale, (T*)dqkv)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_assemble_q_slab_inplace(const float* dql, const void* slab, int slabs, int nbags, int nh, int n,
                                              float scale, void* dqkv, void* stream) {
  TM_REQUIRE(n > 0 && n % NL == 0 && nh > 0 && nh <= 8 && slabs > 0, "assemble_q_slab_inplace: bad shape");
  TM_REQUIRE(dql && slab && dqkv && ((uintptr_t)dqkv % 16) == 0, "assemble_q_slab_inplace: null / misaligned operand");
  assemble_q_slab_kernel<bf16, true><<<dim3(NL, nbags), AQ_THREADS, 0, (hipStream_t)stream>>>(
      nullptr, -1, dql, (const bf16*)slab, slabs, (long long)nbags * nh * NL * DH, n, n / NL, nh, scale, (bf16*)dqkv);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_assemble_q(int dtype, const float* dq, int dq_row, const float* dql_a, const float* dql_b,
                                 int nbags, int nh, int n, float scale, void* dqkv, void* stream) {
  TM_REQUIRE(n % NL == 0, "assemble_q: n must be a multiple of 256");
  const long long items = (long long)n * nh * DH / 8;
  TM_DTYPE_DISPATCH(dtype, (assemble_q_kernel<T><<<dim3((unsigned)((items + 255) / 256), nbags), 256, 0,
                                                    (hipStream_t)stream>>>(dq, dq_row, dql_a, dql_b, n, n / NL, nh,
                                                                           scale, (T*)dqkv)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_nys_assemble_dqkv(int dtype, const float* dq, const float* dql, const float* dk, const float* dkl,
                                    const float* dv, int nbags, int nh, int n, float scale, void* dqkv,
                                    void* stream) {
  TM_REQUIRE(n % NL == 0, "assemble_dqkv: n must be a multiple of 256");
  const long long items = (long long)n * 3 * nh * DH / 8;
  TM_DTYPE_DISPATCH(dtype, (assemble_dqkv_kernel<T><<<dim3((unsigned)((items + 255) / 256), nbags), 256, 0,
                                                       (hipStream_t)stream>>>(
                               dq, dql, dk, dkl, dv, n, n / NL, nh, scale, (T*)dqkv)));
  TM_CHECK_LAUNCH();
  return 0;
}
