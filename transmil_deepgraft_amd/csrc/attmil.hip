// AttMIL gated attention pooling (code/models/AttMIL.py:88-110), fp32, the non-GEMM half:
//   a_i   = w . (tanh(Zv_i) * sigmoid(Zu_i)) + b        Z = H [Wv;Wu]^T + [bv;bu] (the caller's GEMM)
//   p     = softmax_N(a)                                 (:101-104)
//   M     = sum_i p_i H_i ;  logits = M Wc^T + bc         (:105-106)
// and its backward down to dZ (the caller's GEMMs take dZ to dH, d[Wv;Wu], d[bv;bu]):
//   dM = dl Wc ; dWc = dl^T M ; dbc = dl
//   dp_i = H_i . dM ; da_i = p_i (dp_i - sum_j p_j dp_j)
//   dZv = da w sig (1 - tanh^2) ; dZu = da w tanh sig (1 - sig) ; dw = sum_i da tanh sig ; db = sum_i da
//   dH_i = p_i dM   (the GEMM then adds dZ [Wv;Wu])
// HBM-bound row passes over H [N, L] and Z [N, 2D]; every reduction is a fixed-order tree, so
// results are deterministic run to run.
#include "common.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int POOL_ROWS = 64;     // rows of H per pooling / backward-row block

TM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
TM_DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// block-wide sum / max of one value per thread (blockDim.x multiple of 64, <= 1024)
template <bool MAX>
TM_DEV float block_reduce(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o);
    v = MAX ? fmaxf(v, u) : v + u;
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < nw; ++i) r = MAX ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

// one wave per instance row: a_i = sum_d tanh(Z[i][d]) sigmoid(Z[i][D+d]) w[d] + b
__global__ void __launch_bounds__(256) score_kernel(const float* __restrict__ Z, int N, int D,
                                                    const float* __restrict__ w, const float* __restrict__ b,
                                                    float* __restrict__ a) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= N) return;
  const float* z = Z + (size_t)i * 2 * D;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64) acc += tanhf(z[d]) * sigmoidf_(z[D + d]) * w[d];
  acc = wave_sum(acc);
  if (lane == 0) a[i] = acc + b[0];
}

// softmax statistics over all N scores: stats = {max, sum exp(a - max)}; one block
__global__ void __launch_bounds__(1024) stats_kernel(const float* __restrict__ a, int N, float* __restrict__ stats) {
  __shared__ float red[16];
  float m = -INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) m = fmaxf(m, a[i]);
  m = block_reduce<true>(m, red);
  float s = 0.f;
  for (int i = threadIdx.x; i < N; i += blockDim.x) s += __expf(a[i] - m);
  s = block_reduce<false>(s, red);
  if (threadIdx.x == 0) {
    stats[0] = m;
    stats[1] = s;
  }
}

// partial[blk][c] = sum over this block's rows of p_i H[i][c]; also p_i; block = L/4 threads (float4 columns)
__global__ void pool_partial_kernel(const float* __restrict__ a, const float* __restrict__ stats,
                                    const float* __restrict__ H, int N, int L, float* __restrict__ p,
                                    float* __restrict__ partial) {
  const int r0 = blockIdx.x * POOL_ROWS, r1 = min(N, r0 + POOL_ROWS), t = threadIdx.x;
  const float m = stats[0], inv = 1.f / stats[1];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = r0; i < r1; ++i) {
    const float pi = __expf(a[i] - m) * inv;
    if (t == 0) p[i] = pi;
    const f32x4 h = *(const f32x4*)(H + (size_t)i * L + 4 * t);
    acc += pi * h;
  }
  *(f32x4*)(partial + (size_t)blockIdx.x * L + 4 * t) = acc;
}

// M[c] = sum_blk partial[blk][c] ; logits[k] = M . Wc[k] + bc[k]; one block of 256
__global__ void __launch_bounds__(256) pool_final_kernel(const float* __restrict__ partial, int nblk, int L,
                                                         const float* __restrict__ Wc, const float* __restrict__ bc,
                                                         int C, float* __restrict__ M, float* __restrict__ logits) {
  extern __shared__ float sm[];   // L floats of M + 4 reduction slots
  float* red = sm + L;
  for (int c = threadIdx.x; c < L; c += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += partial[(size_t)k * L + c];
    sm[c] = s;
    M[c] = s;
  }
  __syncthreads();
  for (int k = 0; k < C; ++k) {
    float s = 0.f;
    for (int c = threadIdx.x; c < L; c += blockDim.x) s += sm[c] * Wc[(size_t)k * L + c];
    s = block_reduce<false>(s, red);
    if (threadIdx.x == 0) logits[k] = s + bc[k];
  }
}

// dM = dl Wc, dWc = dl^T M, dbc = dl; one block of 256
__global__ void __launch_bounds__(256) bwd_head_kernel(const float* __restrict__ dl, const float* __restrict__ M,
                                                       const float* __restrict__ Wc, int C, int L,
                                                       float* __restrict__ dM, float* __restrict__ dWc,
                                                       float* __restrict__ dbc) {
  for (int c = threadIdx.x; c < L; c += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < C; ++k) {
      s += dl[k] * Wc[(size_t)k * L + c];
      dWc[(size_t)k * L + c] = dl[k] * M[c];
    }
    dM[c] = s;
  }
  if (threadIdx.x < C) dbc[threadIdx.x] = dl[threadIdx.x];
}

// one wave per row: dp_i = H_i . dM ; part[blk] = sum over the block's 4 rows of p_i dp_i
__global__ void __launch_bounds__(256) bwd_dp_kernel(const float* __restrict__ H, const float* __restrict__ dM,
                                                     const float* __restrict__ p, int N, int L,
                                                     float* __restrict__ dp, float* __restrict__ part) {
  __shared__ float red[4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, i = blockIdx.x * 4 + wv;
  float v = 0.f;
  if (i < N) {
    const float* h = H + (size_t)i * L;
    float s = 0.f;
    for (int c = 4 * lane; c < L; c += 256) {
      const f32x4 x = *(const f32x4*)(h + c), g = *(const f32x4*)(dM + c);
      s += x[0] * g[0] + x[1] * g[1] + x[2] * g[2] + x[3] * g[3];
    }
    s = wave_sum(s);
    if (lane == 0) dp[i] = s;
    v = p[i] * s;
  }
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// POOL_ROWS rows per block, one wave per row at a time: dZ, dH = p dM, and per-block dw / db partials
__global__ void __launch_bounds__(256) bwd_rows_kernel(const float* __restrict__ Z, const float* __restrict__ w,
                                                       const float* __restrict__ p, const float* __restrict__ dp,
                                                       const float* __restrict__ part, int npart,
                                                       const float* __restrict__ dM, int N, int D, int L,
                                                       float* __restrict__ dZ, float* __restrict__ dH,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part) {
  extern __shared__ float sm[];   // 4 x D dw partials + 4 db + 4 reduction slots
  float* red = sm + 4 * D + 4;
  // S = sum_j p_j dp_j, summed in the same order by every block
  float s = 0.f;
  for (int k = threadIdx.x; k < npart; k += blockDim.x) s += part[k];
  const float S = block_reduce<false>(s, red);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = blockIdx.x * POOL_ROWS, r1 = min(N, r0 + POOL_ROWS);
  for (int d = lane; d < D; d += 64) sm[wv * D + d] = 0.f;
  float dbacc = 0.f;
  for (int i = r0 + wv; i < r1; i += 4) {
    const float pi = p[i], da = pi * (dp[i] - S);
    const float* z = Z + (size_t)i * 2 * D;
    float* gz = dZ + (size_t)i * 2 * D;
    for (int d = lane; d < D; d += 64) {
      const float t = tanhf(z[d]), sg = sigmoidf_(z[D + d]), wd = w[d];
      gz[d] = da * wd * sg * (1.f - t * t);
      gz[D + d] = da * wd * t * sg * (1.f - sg);
      sm[wv * D + d] += da * t * sg;
    }
    dbacc += da;
    float* gh = dH + (size_t)i * L;
    for (int c = 4 * lane; c < L; c += 256) *(f32x4*)(gh + c) = pi * *(const f32x4*)(dM + c);
  }
  if (lane == 0) sm[4 * D + wv] = dbacc;
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x)
    dw_part[(size_t)blockIdx.x * D + d] = sm[d] + sm[D + d] + sm[2 * D + d] + sm[3 * D + d];
  if (threadIdx.x == 0) db_part[blockIdx.x] = sm[4 * D] + sm[4 * D + 1] + sm[4 * D + 2] + sm[4 * D + 3];
}

// dw[d] = sum_blk dw_part[blk][d] ; db = sum_blk db_part[blk]; one block of 256
__global__ void __launch_bounds__(256) bwd_reduce_kernel(const float* __restrict__ dw_part,
                                                         const float* __restrict__ db_part, int nblk, int D,
                                                         float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[4];
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += dw_part[(size_t)k * D + d];
    dw[d] = s;
  }
  float s = 0.f;
  for (int k = threadIdx.x; k < nblk; k += blockDim.x) s += db_part[k];
  s = block_reduce<false>(s, red);
  if (threadIdx.x == 0) db[0] = s;
}

int nblk_rows(int N) { return (N + POOL_ROWS - 1) / POOL_ROWS; }

}  // namespace

extern "C" long long tm_attmil_fwd_workspace(int N, int L) {
  return (long long)(4 + (size_t)nblk_rows(N) * L) * sizeof(float);
}

extern "C" int tm_attmil_fwd(const float* Z, const float* H, const float* w, const float* b, const float* Wc,
                             const float* bc, int N, int L, int D, int C, float* work, float* a, float* p, float* M,
                             float* logits, void* stream) {
  TM_REQUIRE(N >= 1 && D >= 1 && C >= 1, "attmil_fwd: empty shape");
  TM_REQUIRE(L % 4 == 0 && L / 4 <= 1024, "attmil_fwd: L must be a multiple of 4, <= 4096");
  hipStream_t st = (hipStream_t)stream;
  float* stats = work;
  float* partial = work + 4;
  const int nblk = nblk_rows(N);
  score_kernel<<<(N + 3) / 4, 256, 0, st>>>(Z, N, D, w, b, a);
  stats_kernel<<<1, 1024, 0, st>>>(a, N, stats);
  pool_partial_kernel<<<nblk, L / 4, 0, st>>>(a, stats, H, N, L, p, partial);
  pool_final_kernel<<<1, 256, (L + 4) * sizeof(float), st>>>(partial, nblk, L, Wc, bc, C, M, logits);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_attmil_bwd_workspace(int N, int L, int D) {
  (void)L;
  return (long long)((size_t)(N + 3) / 4 + N + (size_t)nblk_rows(N) * (D + 1) + 4) * sizeof(float);
}

extern "C" int tm_attmil_bwd(const float* Z, const float* H, const float* w, const float* p, const float* M,
                             const float* Wc, const float* dlogits, int N, int L, int D, int C, float* work,
                             float* dZ, float* dH, float* dM, float* dw, float* db, float* dWc, float* dbc,
                             void* stream) {
  TM_REQUIRE(N >= 1 && D >= 1 && C >= 1 && C <= 256, "attmil_bwd: bad shape");
  TM_REQUIRE(L % 4 == 0, "attmil_bwd: L must be a multiple of 4");
  hipStream_t st = (hipStream_t)stream;
  const int npart = (N + 3) / 4, nblk = nblk_rows(N);
  float* part = work;                       // [npart] p_i dp_i partial sums
  float* dp = part + npart;                 // [N]
  float* dw_part = dp + N;                  // [nblk][D]
  float* db_part = dw_part + (size_t)nblk * D;   // [nblk]
  bwd_head_kernel<<<1, 256, 0, st>>>(dlogits, M, Wc, C, L, dM, dWc, dbc);
  bwd_dp_kernel<<<npart, 256, 0, st>>>(H, dM, p, N, L, dp, part);
  bwd_rows_kernel<<<nblk, 256, (4 * D + 8) * sizeof(float), st>>>(Z, w, p, dp, part, npart, dM, N, D, L, dZ, dH,
                                                                 dw_part, db_part);
  bwd_reduce_kernel<<<1, 256, 0, st>>>(dw_part, db_part, nblk, D, dw, db);
  TM_CHECK_LAUNCH();
  return 0;
}
