// MFMA GEMM with fused epilogues for the dense d_model projections of TransMIL:
// _fc1 (+GELU), NystromAttention.to_qkv (+head-major scatter, q scale),
// to_out (+bias, dropout, residual add into the fp32 residual stream) and the
// backward data/weight products.  Replaces the torch Linear call sites
// code/models/TransMIL.py:128-133 (fc1) and the to_qkv / to_out Linears of the
// third-party NystromAttention.
//
//   C[m, n] = epilogue( alpha * sum_k A(m,k) * B(k,n) )
//   A(m,k) = A_T ? A[k*lda + m] : A[m*lda + k]
//   B(k,n) = B_KN ? B[k*ldb + n] : B[n*ldb + k]
//
// Block tile 128x128, 4 waves in 2x2, each wave 64x64 = 2x2 MFMA 32x32 tiles.
// K staged through LDS in 64-byte rows (+16 B pad: conflict-free ds_read_b128
// for the 16-lane groups), register double buffering.  Split-K writes fp32
// slabs that tm_splitk_reduce sums in a fixed order (bitwise reproducible).
#include "common.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int BM = 128, BN = 128;

template <typename T> struct Tile {
  static constexpr int E = 16 / sizeof(T);            // elements per 16-B chunk
  static constexpr int BK = 64 / sizeof(T);           // 32 bf16, 16 f32
  static constexpr int ROW = BK + E;                  // LDS row (elements), 80 B
  static constexpr int KSTEPS = BK / 16;
};

template <typename T> union Chunk { f32x4 raw; T e[16 / sizeof(T)]; };

// Non-transposed operand: rows r0.., k contiguous.  Chunk c: row c>>2, col (c&3)*E.
template <typename T>
TM_DEV void load_rows(Chunk<T> (&st)[2], const T* X, int ld, int r0, int rmax, int k0, int kend, int tid) {
  constexpr int E = Tile<T>::E;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    const int row = c >> 2, col = (c & 3) * E;
    const int gr = r0 + row, gk = k0 + col;
    if (gr < rmax && gk + E <= kend) {
      st[i].raw = *(const f32x4*)(X + (size_t)gr * ld + gk);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e)
        st[i].e[e] = (gr < rmax && gk + e < kend) ? X[(size_t)gr * ld + gk + e] : from_f<T>(0.f);
    }
  }
}
template <typename T>
TM_DEV void store_rows(T* S, const Chunk<T> (&st)[2], int tid) {
  constexpr int E = Tile<T>::E, ROW = Tile<T>::ROW;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    *(f32x4*)(S + (c >> 2) * ROW + (c & 3) * E) = st[i].raw;
  }
}
// Transposed operand: global [k][m] (m contiguous).  Chunk c: k-row c / CPR, m-col (c % CPR)*E.
template <typename T>
TM_DEV void load_cols(Chunk<T> (&st)[2], const T* X, int ld, int m0, int mmax, int k0, int kend, int tid) {
  constexpr int E = Tile<T>::E, CPR = BM / E;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    const int kr = c / CPR, mc = (c % CPR) * E;
    const int gk = k0 + kr, gm = m0 + mc;
    if (gk < kend && gm + E <= mmax) {
      st[i].raw = *(const f32x4*)(X + (size_t)gk * ld + gm);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e)
        st[i].e[e] = (gk < kend && gm + e < mmax) ? X[(size_t)gk * ld + gm + e] : from_f<T>(0.f);
    }
  }
}
template <typename T>
TM_DEV void store_cols(T* S, const Chunk<T> (&st)[2], int tid) {
  constexpr int E = Tile<T>::E, CPR = BM / E, ROW = Tile<T>::ROW;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    const int kr = c / CPR, mc = (c % CPR) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) S[(mc + e) * ROW + kr] = st[i].e[e];
  }
}

template <typename OutT>
TM_DEV void put(OutT* p, float v) { *p = from_f<OutT>(v); }

// One output element of the GEMM epilogue (kept out of line of the unrolled
// accumulator loops so the accumulators stay in registers).
template <typename OutT>
TM_DEV void epilogue_elem(OutT* __restrict__ C, const tm_gemm_args& g, int m, int n, float v) {
  if (m >= g.M || n >= g.N) return;
  if (g.mode == TM_EPI_SPLITK) {  // fp32 slab [split][M][N]
    ((float*)C)[((size_t)blockIdx.z * g.M + m) * g.N + n] = v;
    return;
  }
  v *= g.alpha;
  if (g.bias) v += g.bias[n];
  if (g.mode == TM_EPI_QKV) {
    const int bag = m / g.seq, t = m % g.seq;
    const int inner = g.nh * g.dh;
    const int which = n / inner, hh = (n % inner) / g.dh, d = n % g.dh;
    if (which == 0) v *= g.qscale;
    const size_t dst = (((size_t)which * g.nbags * g.nh + (size_t)bag * g.nh + hh) * g.seq + t) * g.dh + d;
    put(C + dst, v);
    return;
  }
  if (g.pre) put((OutT*)g.pre + (size_t)m * g.ld_pre + n, v);
  if (g.gelu) v = gelu_erf(v);
  int row = m, dup_row = -1;
  if (g.grp_in > 0) {
    const int bag = m / g.grp_in, t = m % g.grp_in - g.skip;
    if (t < 0) return;
    row = bag * g.grp_out + g.out_off + t;
    if (t < g.dup_n) dup_row = bag * g.grp_out + g.dup_off + t;
  }
  if (g.drop_p > 0.f) {
    const float u = dropout_u01(g.seed, (uint32_t)row, (uint32_t)n);
    v = (u >= g.drop_p) ? v * g.drop_scale : 0.f;
  }
  const size_t off = (size_t)row * g.ldc + n;
  if (g.resid) v += g.resid[off];
  if (g.accumulate) v += to_f(C[off]);
  put(C + off, v);
  if (dup_row >= 0) put(C + (size_t)dup_row * g.ldc + n, v);
}

template <typename T, typename OutT, bool A_T, bool B_KN>
__global__ __launch_bounds__(256) void gemm_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                   OutT* __restrict__ C, tm_gemm_args g) {
  using TT = Tile<T>;
  constexpr int ROW = TT::ROW, BK = TT::BK;
  __shared__ __attribute__((aligned(16))) T As[2][BM * ROW];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * ROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){};

  Chunk<T> sa[2], sb[2];
  auto gload = [&](int k0) {
    if constexpr (A_T) load_cols(sa, A, g.lda, m0, g.M, k0, kend, tid);
    else load_rows(sa, A, g.lda, m0, g.M, k0, kend, tid);
    if constexpr (B_KN) load_cols(sb, B, g.ldb, n0, g.N, k0, kend, tid);
    else load_rows(sb, B, g.ldb, n0, g.N, k0, kend, tid);
  };
  auto lstore = [&](int buf) {
    if constexpr (A_T) store_cols(As[buf], sa, tid); else store_rows(As[buf], sa, tid);
    if constexpr (B_KN) store_cols(Bs[buf], sb, tid); else store_rows(Bs[buf], sb, tid);
  };

  if (nk > 0) {
    gload(kbeg);
    lstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kbeg + (kt + 1) * BK);
    const T* as = As[cur];
    const T* bs = Bs[cur];
#pragma unroll
    for (int s = 0; s < TT::KSTEPS; ++s) {
      vec8<T> af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = load8(as + (wm * 64 + i * 32 + l32) * ROW + s * 16 + 8 * h);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = load8(bs + (wn * 64 + j * 32 + l32) * ROW + s * 16 + 8 * h);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mma16(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  auto tile_epi = [&](const f32x16& a, int i, int j) {
    const int n = n0 + wn * 64 + j * 32 + l32;
    const int mb = m0 + wm * 64 + i * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) epilogue_elem<OutT>(C, g, mb + acc_row(r, h), n, a[r]);
  };
  tile_epi(acc[0][0], 0, 0);
  tile_epi(acc[0][1], 0, 1);
  tile_epi(acc[1][0], 1, 0);
  tile_epi(acc[1][1], 1, 1);
}

template <typename T, typename OutT>
int launch_t(const void* A, const void* B, void* C, const tm_gemm_args& g, hipStream_t st) {
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, g.splits);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
  OutT* c = (OutT*)C;
#define TM_GEMM_CASE(AT, BKN) \
  if (g.a_trans == AT && g.b_kn == BKN) { gemm_kernel<T, OutT, AT, BKN><<<grid, 256, 0, st>>>(a, b, c, g); TM_CHECK_LAUNCH(); return 0; }
  TM_GEMM_CASE(0, 0) TM_GEMM_CASE(0, 1) TM_GEMM_CASE(1, 0) TM_GEMM_CASE(1, 1)
#undef TM_GEMM_CASE
  tm_set_error("gemm: bad transpose flags");
  return 1;
}

__global__ void splitk_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out, int splits,
                                     size_t count, float alpha, int accumulate) {
  const size_t i4 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 * 4 >= count) return;
  if (i4 * 4 + 4 <= count) {
    f32x4 s = *(const f32x4*)(slab + i4 * 4);
    for (int z = 1; z < splits; ++z) s += *(const f32x4*)(slab + (size_t)z * count + i4 * 4);
    s *= alpha;
    if (accumulate) s += *(f32x4*)(out + i4 * 4);
    *(f32x4*)(out + i4 * 4) = s;
  } else {
    for (size_t i = i4 * 4; i < count; ++i) {
      float s = slab[i];
      for (int z = 1; z < splits; ++z) s += slab[(size_t)z * count + i];
      s *= alpha;
      if (accumulate) s += out[i];
      out[i] = s;
    }
  }
}

// column sums of a [rows, cols] matrix into fp32 partials: grid (ceil(cols/64), nchunks)
template <typename T>
__global__ void colsum_partial_kernel(const T* __restrict__ X, int rows, int cols, int ld, int rows_per_chunk,
                                      float* __restrict__ part) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sub = threadIdx.x >> 6;  // 4 row phases
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(rows, r0 + rows_per_chunk);
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < cols)
    for (int r = r0 + sub; r < r1; r += 4) s += to_f(X[(size_t)r * ld + c]);
  red[sub][threadIdx.x & 63] = s;
  __syncthreads();
  if (sub == 0 && c < cols)
    part[(size_t)blockIdx.y * cols + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

}  // namespace

extern "C" int tm_gemm(const void* A, const void* B, void* C, const tm_gemm_args* g, void* stream) {
  TM_REQUIRE(g && A && B && C, "gemm: null argument");
  TM_REQUIRE(g->M >= 0 && g->N >= 0 && g->K >= 0 && g->splits >= 1, "gemm: bad shape");
  TM_REQUIRE(g->mode != TM_EPI_SPLITK || g->c_dtype == TM_F32, "gemm: split-K slabs are fp32");
  TM_REQUIRE(g->k_per_split > 0, "gemm: k_per_split must be > 0");
  TM_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "gemm: operands must be 16-B aligned");
  const int E = g->ab_dtype == TM_BF16 ? 8 : 4;
  TM_REQUIRE(g->lda % E == 0 && g->ldb % E == 0, "gemm: leading dimensions must be multiples of 16 B");
  if (g->M == 0 || g->N == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (g->ab_dtype == TM_BF16) {
    if (g->c_dtype == TM_BF16) return launch_t<bf16, bf16>(A, B, C, *g, st);
    return launch_t<bf16, float>(A, B, C, *g, st);
  }
  TM_REQUIRE(g->ab_dtype == TM_F32, "gemm: ab_dtype");
  if (g->c_dtype == TM_BF16) return launch_t<float, bf16>(A, B, C, *g, st);
  return launch_t<float, float>(A, B, C, *g, st);
}

extern "C" int tm_splitk_reduce(const float* slab, float* out, int splits, long long count, float alpha,
                                int accumulate, void* stream) {
  TM_REQUIRE(slab && out && splits >= 1 && count >= 0, "splitk_reduce: bad args");
  if (count == 0) return 0;
  const size_t n4 = ((size_t)count + 3) / 4;
  splitk_reduce_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, (hipStream_t)stream>>>(slab, out, splits, (size_t)count,
                                                                                    alpha, accumulate);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_colsum_workspace(int rows, int cols, int rows_per_chunk) {
  const int nchunk = (rows + rows_per_chunk - 1) / rows_per_chunk;
  return (long long)nchunk * cols * (long long)sizeof(float);
}

// out[c] (+)= sum_r X[r, c]; deterministic two-level sum through `work`
extern "C" int tm_colsum(const void* X, int dtype, int rows, int cols, int ld, int rows_per_chunk, float* work,
                         float* out, int accumulate, void* stream) {
  TM_REQUIRE(X && work && out && rows_per_chunk > 0, "colsum: bad args");
  const int nchunk = (rows + rows_per_chunk - 1) / rows_per_chunk;
  dim3 grid((cols + 63) / 64, nchunk);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16)
    colsum_partial_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)X, rows, cols, ld, rows_per_chunk, work);
  else
    colsum_partial_kernel<float><<<grid, 256, 0, st>>>((const float*)X, rows, cols, ld, rows_per_chunk, work);
  TM_CHECK_LAUNCH();
  return tm_splitk_reduce(work, out, nchunk, cols, 1.0f, accumulate, stream);
}
