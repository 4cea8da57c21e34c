// Rows of the NystromAttention `return_attn` product without the n x n matrix.
//
// The reference returns attn1 @ pinv(attn2) @ attn3 ([B, h, n, n], SURVEY.md App. A eq. 11;
// code/models/TransMIL.py:47,209-210) and its consumers read ONE row of it:
// cls_attention[0, :, padding+1, padding+1:padding+1+H] (code/visualize_mil.py:580-581,
// visualize_feat_lvl.py:569, gradcam_sus.py:571).  Row r of head bh is
//   out[t] = sum_j w_j exp(ql_j . k_t - lse3_j),   w = softmax(q_r kl^T) Z
// i.e. O(h (m^2 + m n)) work instead of O(h n^2 m), with the forward's own factors:
// q, k (T, q pre-scaled by dim_head^-0.5), landmarks ql / kl (fp32), Z = pinv(attn2) (fp32)
// and attn3's log-sum-exp rows lse3 (fp32).  fp32 arithmetic throughout.
#include "common.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int NLR = 256;  // landmarks
constexpr int DHR = 64;   // dim_head

// grid (n / 256, nbh), block 256: one token per thread.  Each block recomputes w for its
// head (256 x 64 + 256 x 256 MACs, negligible next to its 256 x 256 x 64 token dots).
template <typename T>
__global__ __launch_bounds__(256) void attn_row_kernel(const T* __restrict__ q, const T* __restrict__ k,
                                                       const float* __restrict__ ql, const float* __restrict__ kl,
                                                       const float* __restrict__ z, const float* __restrict__ lse3,
                                                       int n, int row, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float qls[NLR * DHR];  // 64 KB
  __shared__ float a1[NLR], w[NLR], lse[NLR], red[8];
  const int tid = threadIdx.x, bh = blockIdx.y;
  const size_t hq = (size_t)bh * n * DHR;
  const size_t hl = (size_t)bh * NLR * DHR;
  // attn1 row r: softmax over the 256 landmarks (thread j = landmark j)
  float s = 0.f;
  {
    const T* qr = q + hq + (size_t)row * DHR;
    const float* kj = kl + hl + (size_t)tid * DHR;
#pragma unroll 8
    for (int d = 0; d < DHR; ++d) s = fmaf(to_f(qr[d]), kj[d], s);
  }
  float m = wave_max(s);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float e = expf(s - m);
  float sum = wave_sum(e);
  if ((tid & 63) == 0) red[4 + (tid >> 6)] = sum;
  __syncthreads();
  sum = (red[4] + red[5]) + (red[6] + red[7]);
  a1[tid] = e / sum;
  lse[tid] = lse3[(size_t)bh * NLR + tid];
  // ql of this head -> LDS (16 B per lane)
  for (int c = tid; c < NLR * DHR / 4; c += 256)
    *(f32x4*)(qls + c * 4) = *(const f32x4*)(ql + hl + (size_t)c * 4);
  __syncthreads();
  // w = attn1_row Z  (thread i = column i of Z)
  {
    const float* zh = z + (size_t)bh * NLR * NLR;
    float acc = 0.f;
#pragma unroll 8
    for (int j = 0; j < NLR; ++j) acc = fmaf(a1[j], zh[(size_t)j * NLR + tid], acc);
    w[tid] = acc;
  }
  __syncthreads();
  // out[t] = sum_j w_j exp(ql_j . k_t - lse3_j)
  const int t = blockIdx.x * 256 + tid;
  if (t >= n) return;
  float kr[DHR];
  {
    const T* kt = k + hq + (size_t)t * DHR;
#pragma unroll
    for (int d = 0; d < DHR; ++d) kr[d] = to_f(kt[d]);
  }
  float acc = 0.f;
  for (int j = 0; j < NLR; ++j) {
    const float* qj = qls + j * DHR;  // every lane reads the same row: LDS broadcast
    float d0 = 0.f, d1 = 0.f;
#pragma unroll
    for (int d = 0; d < DHR; d += 8) {
      const f32x4 a = *(const f32x4*)(qj + d), b = *(const f32x4*)(qj + d + 4);
      d0 = fmaf(a[0], kr[d], d0); d1 = fmaf(a[1], kr[d + 1], d1);
      d0 = fmaf(a[2], kr[d + 2], d0); d1 = fmaf(a[3], kr[d + 3], d1);
      d0 = fmaf(b[0], kr[d + 4], d0); d1 = fmaf(b[1], kr[d + 5], d1);
      d0 = fmaf(b[2], kr[d + 6], d0); d1 = fmaf(b[3], kr[d + 7], d1);
    }
    acc = fmaf(w[j], expf((d0 + d1) - lse[j]), acc);
  }
  out[(size_t)bh * n + t] = acc;
}

}  // namespace

#define TM_DTYPE_DISPATCH(dt, CALL)                               \
  if ((dt) == TM_BF16) { using T = bf16; CALL; }                  \
  else if ((dt) == TM_F32) { using T = float; CALL; }             \
  else { tm_set_error("attn_row: dtype must be TM_F32 or TM_BF16"); return 1; }

extern "C" int tm_nys_attn_row(int dtype, const void* q, const void* k, const float* ql, const float* kl,
                               const float* z, const float* lse3, int nbh, int n, int row, float* out,
                               void* stream) {
  TM_REQUIRE(q && k && ql && kl && z && lse3 && out, "attn_row: null pointer");
  TM_REQUIRE(nbh > 0 && n > 0 && n % 256 == 0, "attn_row: n must be a positive multiple of 256");
  TM_REQUIRE(row >= 0 && row < n, "attn_row: row out of range");
  const dim3 grid(n / 256, nbh);
  hipStream_t st = (hipStream_t)stream;
  TM_DTYPE_DISPATCH(dtype, (attn_row_kernel<T><<<grid, 256, 0, st>>>((const T*)q, (const T*)k, ql, kl, z, lse3, n,
                                                                      row, out)));
  TM_CHECK_LAUNCH();
  return 0;
}
