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
// Block tile 128x128, 4 waves in 2x2, each wave 64x64 = 2x2 v_mfma 32x32 tiles.
// K staged through LDS in 128-byte slices (BK = 64 bf16 / 32 f32), register
// double buffering, 16 MFMAs per wave between barriers.
//   * k-contiguous operand: LDS [row][BK + 16 B]  -> ds_read_b128 fragments
//     (144 B rows: the 16-lane groups hit 16 distinct 16-B slots).
//   * k-strided operand (weight gradients, X^T dY), bf16: the tile is stored
//     as it lies in HBM, LDS [k][128 + 32] (320 B rows, 64 distinct banks per
//     32-lane half), and read with ds_read_b64_tr_b16, the gfx950 transposing
//     LDS read: two 4(k) x 16(m) blocks form one 8-deep fragment.  No scalar
//     transposes anywhere.  (fp32 parity mode transposes on the LDS write.)
// Split-K writes fp32 slabs that tm_splitk_reduce sums in a fixed order
// (bitwise reproducible; no float atomics).
#include "common.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int BM = 128, BN = 128;

template <typename T> struct Tile {
  static constexpr int E = 16 / sizeof(T);             // elements per 16-B chunk
  static constexpr int BK = 128 / sizeof(T);           // 64 bf16, 32 f32: one 128-B slice
  static constexpr int KROW = BK + E;                  // k-contiguous LDS row: 144 B
  static constexpr int TROW = BM + 32;                 // bf16 k-strided LDS row: 320 B
  static constexpr int KSTEPS = BK / 16;
  static constexpr int CHUNKS = BM * BK / E / 256;     // 16-B chunks per thread per operand (4)
};

template <typename T> union Chunk { f32x4 raw; T e[16 / sizeof(T)]; };

// k-contiguous operand rows r0.. : chunk c -> row c / (BK/E), col (c % (BK/E)) * E
template <typename T>
TM_DEV void load_rows(Chunk<T> (&st)[Tile<T>::CHUNKS], const T* X, int ld, int r0, int rmax, int k0, int kend,
                      int tid) {
  constexpr int E = Tile<T>::E, CPR = Tile<T>::BK / E;
#pragma unroll
  for (int i = 0; i < Tile<T>::CHUNKS; ++i) {
    const int c = tid + 256 * i;
    const int row = c / CPR, col = (c % CPR) * E;
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
TM_DEV void store_rows(T* S, const Chunk<T> (&st)[Tile<T>::CHUNKS], int tid) {
  constexpr int E = Tile<T>::E, CPR = Tile<T>::BK / E, ROW = Tile<T>::KROW;
#pragma unroll
  for (int i = 0; i < Tile<T>::CHUNKS; ++i) {
    const int c = tid + 256 * i;
    *(f32x4*)(S + (c / CPR) * ROW + (c % CPR) * E) = st[i].raw;
  }
}
// k-strided operand: global [k][m] (m contiguous).  chunk c -> k-row c / CPR, m-col (c % CPR) * E
template <typename T>
TM_DEV void load_cols(Chunk<T> (&st)[Tile<T>::CHUNKS], const T* X, int ld, int m0, int mmax, int k0, int kend,
                      int tid) {
  constexpr int E = Tile<T>::E, CPR = BM / E;
#pragma unroll
  for (int i = 0; i < Tile<T>::CHUNKS; ++i) {
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
// bf16: keep the HBM orientation, LDS [k][TROW]; f32: transpose into [m][KROW]
template <typename T>
TM_DEV void store_cols(T* S, const Chunk<T> (&st)[Tile<T>::CHUNKS], int tid) {
  constexpr int E = Tile<T>::E, CPR = BM / E;
#pragma unroll
  for (int i = 0; i < Tile<T>::CHUNKS; ++i) {
    const int c = tid + 256 * i;
    const int kr = c / CPR, mc = (c % CPR) * E;
    if constexpr (sizeof(T) == 2) {
      *(f32x4*)(S + kr * Tile<T>::TROW + mc) = st[i].raw;
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) S[(mc + e) * Tile<T>::KROW + kr] = st[i].e[e];
    }
  }
}

// Fragment of a k-strided bf16 tile via two transposing reads.  Lane l: m = mb + (l&31),
// k = kb + 8*(l>>5) + j.  16-lane group g: lane 4q+p addresses row k0+q, cols m0+4p..+3.
TM_DEV bf16x8 frag_tr(const bf16* S, int mb, int kb, int lane) {
  constexpr int TROW = Tile<bf16>::TROW;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int m = mb + (g & 1) * 16 + 4 * p;
  const int k = kb + 8 * (g >> 1) + q;
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(S + k * TROW + m));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(S + (k + 4) * TROW + m));
  return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <typename T, bool TRANS>
TM_DEV vec8<T> frag(const T* S, int mb, int kb, int lane) {
  if constexpr (TRANS && sizeof(T) == 2) {
    return frag_tr((const bf16*)S, mb, kb, lane);
  } else {
    return load8(S + (mb + (lane & 31)) * Tile<T>::KROW + kb + 8 * (lane >> 5));
  }
}

template <typename T, bool TRANS>
constexpr int tile_elems() {
  return (TRANS && sizeof(T) == 2) ? Tile<T>::BK * Tile<T>::TROW : BM * Tile<T>::KROW;
}

template <typename OutT>
TM_DEV void put(OutT* p, float v) { *p = from_f<OutT>(v); }

template <typename T, typename OutT, bool A_T, bool B_KN>
__global__ __launch_bounds__(256) void gemm_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                   OutT* __restrict__ C, tm_gemm_args g) {
  using TT = Tile<T>;
  constexpr int BK = TT::BK;
  constexpr int AE = tile_elems<T, A_T>(), BE = tile_elems<T, B_KN>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* As0 = (T*)smem;
  T* Bs0 = As0 + 2 * AE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){};

  Chunk<T> sa[TT::CHUNKS], sb[TT::CHUNKS];
  auto gload = [&](int k0) {
    if constexpr (A_T) load_cols(sa, A, g.lda, m0, g.M, k0, kend, tid);
    else load_rows(sa, A, g.lda, m0, g.M, k0, kend, tid);
    if constexpr (B_KN) load_cols(sb, B, g.ldb, n0, g.N, k0, kend, tid);
    else load_rows(sb, B, g.ldb, n0, g.N, k0, kend, tid);
  };
  auto lstore = [&](int buf) {
    if constexpr (A_T) store_cols(As0 + buf * AE, sa, tid); else store_rows(As0 + buf * AE, sa, tid);
    if constexpr (B_KN) store_cols(Bs0 + buf * BE, sb, tid); else store_rows(Bs0 + buf * BE, sb, tid);
  };

  if (nk > 0) {
    gload(kbeg);
    lstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kbeg + (kt + 1) * BK);
    const T* as = As0 + cur * AE;
    const T* bs = Bs0 + cur * BE;
#pragma unroll
    for (int s = 0; s < TT::KSTEPS; ++s) {
      vec8<T> af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag<T, A_T>(as, wm * 64 + i * 32, s * 16, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = frag<T, B_KN>(bs, wn * 64 + j * 32, s * 16, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mma16(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue: row / column bookkeeping hoisted out of the element loop ----------------
  int ncol[2];
  float bcol[2];
  long long cpart[2];   // QKV: column part of the scatter offset
  bool qcol[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + l32;
    ncol[j] = n;
    bcol[j] = (g.bias && n < g.N) ? g.bias[n] : 0.f;
    if (g.mode == TM_EPI_QKV) {
      const int inner = g.nh * g.dh;
      const int which = n / inner, hh = (n % inner) / g.dh, d = n % g.dh;
      cpart[j] = ((long long)which * g.nbags * g.nh + hh) * g.seq * g.dh + d;
      qcol[j] = which == 0;
    } else {
      cpart[j] = 0;
      qcol[j] = false;
    }
  }
  const size_t slab = (size_t)blockIdx.z * g.M * g.N;
  const uint64_t seed = g.drop_p > 0.f ? effective_seed(g.seed, g.seed_ptr) : 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 64 + i * 32 + acc_row(r, h);
      if (m >= g.M) continue;
      if (g.mode == TM_EPI_SPLITK) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (ncol[j] < g.N) ((float*)C)[slab + (size_t)m * g.N + ncol[j]] = acc[i][j][r];
        continue;
      }
      if (g.mode == TM_EPI_QKV) {
        const int bag = m / g.seq, t = m - bag * g.seq;
        const long long rpart = ((long long)bag * g.nh * g.seq + t) * g.dh;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (ncol[j] >= g.N) continue;
          float v = acc[i][j][r] * g.alpha + bcol[j];
          if (qcol[j]) v *= g.qscale;
          put(C + rpart + cpart[j], v);
        }
        continue;
      }
      int row = m, dup_row = -1;
      if (g.grp_in > 0) {
        const int bag = m / g.grp_in, t = m - bag * g.grp_in - g.skip;
        if (t < 0) continue;
        row = bag * g.grp_out + g.out_off + t;
        if (t < g.dup_n) dup_row = bag * g.grp_out + g.dup_off + t;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = ncol[j];
        if (n >= g.N) continue;
        float v = acc[i][j][r] * g.alpha + bcol[j];
        if (g.pre) put((OutT*)g.pre + (size_t)m * g.ld_pre + n, v);
        if (g.gelu) v = gelu_erf(v);
        if (g.drop_p > 0.f) {
          const float u = dropout_u01(seed, (uint32_t)row, (uint32_t)n);
          v = (u >= g.drop_p) ? v * g.drop_scale : 0.f;
        }
        const size_t off = (size_t)row * g.ldc + n;
        if (g.resid) v += g.resid[off];
        if (g.accumulate) v += to_f(C[off]);
        put(C + off, v);
        if (dup_row >= 0) put(C + (size_t)dup_row * g.ldc + n, v);
      }
    }
}

template <typename T, bool A_T, bool B_KN>
constexpr size_t gemm_smem() {
  return 2 * (tile_elems<T, A_T>() + tile_elems<T, B_KN>()) * sizeof(T);
}

template <typename T, typename OutT>
int launch_t(const void* A, const void* B, void* C, const tm_gemm_args& g, hipStream_t st) {
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, g.splits);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
  OutT* c = (OutT*)C;
#define TM_GEMM_CASE(AT, BKN)                                                       \
  if (g.a_trans == AT && g.b_kn == BKN) {                                           \
    constexpr size_t sm = gemm_smem<T, AT, BKN>();                                  \
    tm_allow_smem(gemm_kernel<T, OutT, AT, BKN>, sm);                               \
    gemm_kernel<T, OutT, AT, BKN><<<grid, 256, sm, st>>>(a, b, c, g);               \
    TM_CHECK_LAUNCH();                                                              \
    return 0;                                                                       \
  }
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
#pragma unroll 8
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
    TM_REQUIRE(g->k_per_split % 64 == 0 || g->splits == 1, "gemm: bf16 k_per_split must be a multiple of 64");
    if (g->c_dtype == TM_BF16) return launch_t<bf16, bf16>(A, B, C, *g, st);
    return launch_t<bf16, float>(A, B, C, *g, st);
  }
  TM_REQUIRE(g->ab_dtype == TM_F32, "gemm: ab_dtype");
  TM_REQUIRE(g->k_per_split % 32 == 0 || g->splits == 1, "gemm: f32 k_per_split must be a multiple of 32");
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
