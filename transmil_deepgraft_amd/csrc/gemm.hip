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
#include <new>

#include "common.h"

#include <cstdlib>
#include "../../include/transmil_hip.h"

namespace {

constexpr int BM = 128, BN = 128;
constexpr int EP_ROW = BN + 8;  // epilogue image row (floats): the two lane halves (rows r, r+4) on distinct banks

template <typename T> struct Tile {
  static constexpr int E = 16 / sizeof(T);             // elements per 16-B chunk
  static constexpr int BK = 128 / sizeof(T);           // 64 bf16, 32 f32: one 128-B slice
  static constexpr int KROW = BK + E;                  // k-contiguous LDS row: 144 B
  static constexpr int TROW = BM + 32;                 // bf16 k-strided LDS row: 320 B
  static constexpr int KSTEPS = BK / 16;
  static constexpr int CHUNKS = BM * BK / E / 256;     // 16-B chunks per thread per operand (4)
};

template <typename T> union Chunk { f32x4 raw; T e[16 / sizeof(T)]; };

// Interior tiles (every row and k of the tile in range: a workgroup-uniform test) load
// with no per-chunk bounds branches, so all chunk loads issue back to back and retire
// with one wait; hipcc otherwise branches around each guarded load and waits for it.
template <typename T>
TM_DEV void load_rows_full(Chunk<T> (&st)[Tile<T>::CHUNKS], const T* X, int ld, int r0, int k0, int tid) {
  constexpr int E = Tile<T>::E, CPR = Tile<T>::BK / E;
#pragma unroll
  for (int i = 0; i < Tile<T>::CHUNKS; ++i) {
    const int c = tid + 256 * i;
    st[i].raw = *(const f32x4*)(X + (size_t)(r0 + c / CPR) * ld + k0 + (c % CPR) * E);
  }
}
template <typename T>
TM_DEV void load_cols_full(Chunk<T> (&st)[Tile<T>::CHUNKS], const T* X, int ld, int m0, int k0, int tid) {
  constexpr int E = Tile<T>::E, CPR = BM / E;
#pragma unroll
  for (int i = 0; i < Tile<T>::CHUNKS; ++i) {
    const int c = tid + 256 * i;
    st[i].raw = *(const f32x4*)(X + (size_t)(k0 + c / CPR) * ld + m0 + (c % CPR) * E);
  }
}

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

// Epilogue shared by both main loops: the 2x2 (32x32) accumulators of each of the 4 waves
// (2x2 waves of 64x64) -> LDS [128][EP_ROW] fp32, then 8-column row chunks with 16-B
// loads/stores: bias, pre-activation store, GELU, dropout, residual, accumulate, and the
// TransMIL row maps (grid duplication, QKV head-major scatter, split-K slabs).
// The caller guarantees every wave is past its last read of the staging buffers.
// epilogue kinds: 0 any (runtime mode), 1 plain (alpha, bias, store), 2 QKV scatter, 3 split-K slab
enum { EK_ANY = 0, EK_PLAIN = 1, EK_QKV = 2, EK_SPLITK = 3 };
template <typename OutT, int TBN, int ROWS, int NT, int KIND = EK_ANY>
TM_DEV void gemm_epilogue_rows(const char* smem, OutT* __restrict__ C, const tm_gemm_args& g, int m0, int n0,
                               int split = -1);

// accumulator tile (32x32 at rows rb, cols cb of the block tile) -> epilogue image
TM_DEV void stage_acc(float* ep, const f32x16& acc, int rb, int cb, int lane) {
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int r = 0; r < 16; ++r) ep[(rb + acc_row(r, h)) * EP_ROW + cb + l32] = acc[r];
}

template <typename OutT>
TM_DEV void gemm_epilogue(const f32x16 (&acc)[2][2], char* smem, OutT* __restrict__ C, const tm_gemm_args& g,
                          int m0, int n0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  float* ep = (float*)smem;
  // two passes of 64 rows (the image is 64 x EP_ROW fp32 = 34.8 KB)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wm == half) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) stage_acc(ep, acc[i][j], i * 32, wn * 64 + j * 32, lane);
    }
    __syncthreads();
    gemm_epilogue_rows<OutT, BN, 64, 256>(smem, C, g, m0 + half * 64, n0);
    __syncthreads();
  }
}

// the chunk phase: every thread of the block owns IT 8-column row chunks of the staged tile
// (image rows of TBN + 8 floats), all in the same 8 columns (NT is a multiple of TBN / 8).
// Rolled loops (`unroll 1`): the epilogue runs once per tile, so its code runs from a cold
// instruction cache -- unrolled over IT chunks and every mode it was ~5k instructions and took
// ~8k cycles of a 128 x 128 tile, against ~1.3k for the bare stores (scripts/dev/gemm_epi_probe.py).
// The addend loads (residual / accumulate source) of chunk it + 1 go out before chunk it's
// stores: gfx9 counts stores on vmcnt, so a load issued after a store waits for its write-back.
template <typename OutT, int TBN, int ROWS, int NT, int KIND>
TM_DEV void gemm_epilogue_rows(const char* smem, OutT* __restrict__ C, const tm_gemm_args& g, int m0, int n0,
                               int split) {
  constexpr int CPR = TBN / 8, ROWF = TBN + 8, IT = ROWS * CPR / NT;
  static_assert(ROWS * CPR % NT == 0 && NT % CPR == 0, "epilogue chunk map");
  const int tid = threadIdx.x;
  const float* ep = (const float*)smem;
  const int lc = (tid % CPR) * 8, n = n0 + lc, lr0 = tid / CPR;
  constexpr int LRS = NT / CPR;    // image rows between a thread's chunks
  const int ne = min(8, g.N - n);  // valid columns of this thread's chunks
  if (ne <= 0) return;
  auto chunk = [&](int it, float (&v)[8]) {
    const int lr = lr0 + it * LRS;
    const f32x4 lo = *(const f32x4*)(ep + lr * ROWF + lc), hi = *(const f32x4*)(ep + lr * ROWF + lc + 4);
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3]; v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  };
  if (KIND == EK_SPLITK || (KIND == EK_ANY && g.mode == TM_EPI_SPLITK)) {
    const size_t slab = (size_t)(split < 0 ? (int)blockIdx.z : split) * g.M * g.N;
    if (g.slab_bf16) {   // bf16 slabs: each split's partial rounded once (summed in fp32 by the flush)
      const bool vb = ne == 8 && g.N % 8 == 0;
#pragma unroll 1
      for (int it = 0; it < IT; ++it) {
        const int m = m0 + lr0 + it * LRS;
        if (m >= g.M) break;
        float v[8];
        chunk(it, v);
        bf16* dst = (bf16*)C + slab + (size_t)m * g.N + n;
        if (vb) store8<bf16>(dst, (bf16x8){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5],
                                           (bf16)v[6], (bf16)v[7]});
        else { for (int e = 0; e < ne; ++e) dst[e] = (bf16)v[e]; }
      }
      return;
    }
    const bool vec = ne == 8 && g.N % 4 == 0;
#pragma unroll 1
    for (int it = 0; it < IT; ++it) {
      const int m = m0 + lr0 + it * LRS;
      if (m >= g.M) break;
      float v[8];
      chunk(it, v);
      float* dst = (float*)C + slab + (size_t)m * g.N + n;
      if (vec) {
        *(f32x4*)dst = (f32x4){v[0], v[1], v[2], v[3]};
        *(f32x4*)(dst + 4) = (f32x4){v[4], v[5], v[6], v[7]};
      } else {
        for (int e = 0; e < ne; ++e) dst[e] = v[e];
      }
    }
    return;
  }
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g.bias) {
    if (ne == 8 && ((uintptr_t)g.bias & 15) == 0) { const f32x8 t8 = load8<float>(g.bias + n); for (int e = 0; e < 8; ++e) bv[e] = t8[e]; }
    else { for (int e = 0; e < ne; ++e) bv[e] = g.bias[n + e]; }
  }
  if constexpr (KIND == EK_SPLITK) return;
  if (KIND == EK_QKV || (KIND == EK_ANY && g.mode == TM_EPI_QKV)) {  // 8 columns never straddle a head (dh % 8 == 0, checked on the host)
    const int inner = g.nh * g.dh;
    const int which = n / inner, hh = (n % inner) / g.dh, d = n % g.dh;
    const float qs = which == 0 ? g.qscale : 1.f;
    OutT* base = C + (((long long)which * g.nbags) * g.nh + hh) * g.seq * g.dh + d;
    // (bag, t) of the thread's first row once; later rows step by LRS (< seq) -- no integer
    // division per chunk (it cost ~30 VALU each in the 8-chunk big-tile passes)
    int bag = (m0 + lr0) / g.seq, t = m0 + lr0 - bag * g.seq;
#pragma unroll 1
    for (int it = 0; it < IT; ++it, t += LRS) {
      const int m = m0 + lr0 + it * LRS;
      if (m >= g.M) break;
      while (t >= g.seq) { t -= g.seq; ++bag; }
      OutT* dst = base + (long long)bag * g.nh * g.seq * g.dh + (long long)t * g.dh;
      float v[8];
      chunk(it, v);
      vec8<OutT> o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = from_f<OutT>((v[e] * g.alpha + bv[e]) * qs);
      store8<OutT>(dst, o);
    }
    return;
  }
  if constexpr (KIND == EK_QKV) return;
  if constexpr (KIND == EK_PLAIN) {  // no row map, pre-activation, GELU, dropout or addend
    const bool pvec = ne == 8 && g.ldc % 8 == 0;
#pragma unroll 1
    for (int it = 0; it < IT; ++it) {
      const int m = m0 + lr0 + it * LRS;
      if (m >= g.M) break;
      float v[8];
      chunk(it, v);
      vec8<OutT> o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = from_f<OutT>(v[e] * g.alpha + bv[e]);
      OutT* dst = C + (size_t)m * g.ldc + n;
      if (pvec) store8<OutT>(dst, o);
      else { for (int e = 0; e < ne; ++e) dst[e] = o[e]; }
    }
    return;
  }
  const bool vec = ne == 8 && g.ldc % 8 == 0 && (!g.pre || g.ld_pre % 8 == 0);
  // output row of chunk it (TransMIL grid duplication / padding skip), -1: none
  auto out_row = [&](int it, int& dup) {
    const int m = m0 + lr0 + it * LRS;
    dup = -1;
    if (m >= g.M) return -1;
    if (g.grp_in <= 0) return m;
    const int bag = m / g.grp_in, t = m - bag * g.grp_in - g.skip;
    if (t < 0) return -1;
    if (t < g.dup_n) dup = bag * g.grp_out + g.dup_off + t;
    return bag * g.grp_out + g.out_off + t;
  };
  // the addend (residual, or without one the accumulate source); with both (no caller does)
  // the accumulate source is read at the store
  const float* rsrc = g.resid;
  const OutT* asrc = (g.accumulate && !g.resid) ? C : nullptr;
  const bool acc_late = g.accumulate && g.resid;
  auto load_add = [&](int it, float (&a)[8]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.f;
    int dd;
    const int row = out_row(it, dd);
    if (row < 0) return;
    const size_t off = (size_t)row * g.ldc + n;
    if (rsrc) {
      if (vec) { const f32x8 t8 = load8<float>(rsrc + off); for (int e = 0; e < 8; ++e) a[e] = t8[e]; }
      else { for (int e = 0; e < ne; ++e) a[e] = rsrc[off + e]; }
    } else if (asrc) {
      if (vec) { const vec8<OutT> t8 = load8<OutT>(asrc + off); for (int e = 0; e < 8; ++e) a[e] = to_f(t8[e]); }
      else { for (int e = 0; e < ne; ++e) a[e] = to_f(asrc[off + e]); }
    }
  };
  const bool has_add = rsrc || asrc;
  const uint64_t seed = g.drop_p > 0.f ? effective_seed(g.seed, g.seed_ptr) : 0;
  float av[8];
  if (has_add) load_add(0, av);
#pragma unroll 1
  for (int it = 0; it < IT; ++it) {
    float an[8];
    if (has_add && it + 1 < IT) load_add(it + 1, an);
    int dup;
    const int row = out_row(it, dup);
    if (row >= 0) {
      const size_t off = (size_t)row * g.ldc + n;
      const int m = m0 + lr0 + it * LRS;
      float v[8];
      chunk(it, v);
      // one uniform branch per feature per chunk (a branch per element made this loop
      // VALU-bound: ~7k cycles per tile at four waves per SIMD)
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = v[e] * g.alpha + bv[e];
      vec8<OutT> pre8, out8;
      bf16x8 preb;
      if (g.pre) {
        if (g.pre_bf16) {
#pragma unroll
          for (int e = 0; e < 8; ++e) preb[e] = (bf16)x[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) pre8[e] = from_f<OutT>(x[e]);
        }
      }
      if (g.gelu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = gelu_erf(x[e]);
      }
      if (g.drop_p > 0.f) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float u = dropout_u01(seed, (uint32_t)row, (uint32_t)(n + e));
          x[e] = (u >= g.drop_p) ? x[e] * g.drop_scale : 0.f;
        }
      }
      if (has_add) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] += av[e];
      }
      if (acc_late) {
        for (int e = 0; e < ne; ++e) x[e] += to_f(C[off + e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) out8[e] = from_f<OutT>(x[e]);
      if (vec) {
        if (g.pre) {
          if (g.pre_bf16) store8<bf16>((bf16*)g.pre + (size_t)m * g.ld_pre + n, preb);
          else store8<OutT>((OutT*)g.pre + (size_t)m * g.ld_pre + n, pre8);
        }
        store8<OutT>(C + off, out8);
        if (dup >= 0) store8<OutT>(C + (size_t)dup * g.ldc + n, out8);
      } else {
        for (int e = 0; e < ne; ++e) {
          if (g.pre && g.pre_bf16) ((bf16*)g.pre)[(size_t)m * g.ld_pre + n + e] = preb[e];
          else if (g.pre) ((OutT*)g.pre)[(size_t)m * g.ld_pre + n + e] = pre8[e];
          C[off + e] = out8[e];
          if (dup >= 0) C[(size_t)dup * g.ldc + n + e] = out8[e];
        }
      }
    }
    if (has_add) {
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = an[e];
    }
  }
}

// XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs, so renumber them
// so that each XCD gets a contiguous run of row-major tiles (its row panels of A stay in
// its own L2).  Bijective for any grid size.
TM_DEV void tile_of_block(int& m0, int& n0) {
  const int ntx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int orig = blockIdx.y * ntx + blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  m0 = (id / ntx) * BM;
  n0 = (id % ntx) * BN;
}

// the same renumbering over the whole (x, y, split) grid, splits slowest: an XCD's run of
// workgroups covers one or two splits' K-slices of A and B (split-K launches read each slice's
// panels into one or two L2s instead of all eight).  Bijective for any grid size.
TM_DEV void tile_split_of_block(int& m0, int& n0, int& z) {
  const int ntx = gridDim.x, per = gridDim.x * gridDim.y, nwg = per * gridDim.z;
  const int orig = (blockIdx.z * gridDim.y + blockIdx.y) * ntx + blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  z = id / per;
  const int rr = id - z * per;
  m0 = (rr / ntx) * BM;
  n0 = (rr % ntx) * BN;
}

// NBUF = 2: double-buffered LDS (one barrier per k-tile); NBUF = 1: one LDS buffer, two
// barriers per k-tile, half the LDS -> twice the resident workgroups per CU.
template <typename T, typename OutT, bool A_T, bool B_KN, int NBUF = 2>
__global__ __launch_bounds__(256) void gemm_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                   OutT* __restrict__ C, tm_gemm_args g) {
  using TT = Tile<T>;
  constexpr int BK = TT::BK;
  constexpr int AE = tile_elems<T, A_T>(), BE = tile_elems<T, B_KN>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* As0 = (T*)smem;
  T* Bs0 = As0 + NBUF * AE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int m0, n0;
  tile_of_block(m0, n0);
  const int kbeg = blockIdx.z * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){};

  Chunk<T> sa[TT::CHUNKS], sb[TT::CHUNKS];
  const bool rows_full = m0 + BM <= g.M && n0 + BN <= g.N;
  auto gload = [&](int k0) {
    if (rows_full && k0 + BK <= kend) {
      if constexpr (A_T) load_cols_full(sa, A, g.lda, m0, k0, tid);
      else load_rows_full(sa, A, g.lda, m0, k0, tid);
      if constexpr (B_KN) load_cols_full(sb, B, g.ldb, n0, k0, tid);
      else load_rows_full(sb, B, g.ldb, n0, k0, tid);
    } else {
      if constexpr (A_T) load_cols(sa, A, g.lda, m0, g.M, k0, kend, tid);
      else load_rows(sa, A, g.lda, m0, g.M, k0, kend, tid);
      if constexpr (B_KN) load_cols(sb, B, g.ldb, n0, g.N, k0, kend, tid);
      else load_rows(sb, B, g.ldb, n0, g.N, k0, kend, tid);
    }
  };
  auto lstore = [&](int buf) {
    if constexpr (A_T) store_cols(As0 + buf * AE, sa, tid); else store_rows(As0 + buf * AE, sa, tid);
    if constexpr (B_KN) store_cols(Bs0 + buf * BE, sb, tid); else store_rows(Bs0 + buf * BE, sb, tid);
  };

  if constexpr (NBUF == 1) {
    if (nk > 0) gload(kbeg);
  } else {
    if (nk > 0) {
      gload(kbeg);
      lstore(0);
    }
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NBUF == 1 ? 0 : (kt & 1);
    if constexpr (NBUF == 1) {
      lstore(0);
      __syncthreads();
    }
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
    if (NBUF == 2 && kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  gemm_epilogue<OutT>(acc, smem, C, g, m0, n0);
}

// ---------------------------------------------------------------------------
// bf16 main loop v2: a 4-stage ring of LDS tiles filled by global_load_lds (16 B per
// lane, no VGPR round trip), so three 64-deep k-tiles are in flight while one is
// multiplied.  Per stage: A and B 128 x 64 bf16 images of 16 KB each (128 KB ring,
// one workgroup per CU).  Sync per k-tile: counted `s_waitcnt vmcnt` (never 0 in
// steady state) + raw s_barrier, which also retires the buffer the next prefetch
// overwrites (read in the previous iteration).
// LDS images (bank-clean reads, swizzle applied on the global source address):
//   k-contiguous operand [128 rows][64 k]: 16-B chunk c of row r at slot c ^ ((r >> 1) & 7)
//     -> fragment = one ds_read_b128 per lane (16 consecutive rows hit 16 distinct bank groups)
//   k-strided operand [64 k][128 rows]: chunk c of k-row k at slot c ^ (2 * (k & 3))
//     -> fragment = two ds_read_b64_tr_b16 (4 k-rows x 2 chunks per 16-lane group all distinct)
constexpr int NSTAGE = 4;
constexpr int STAGE_BYTES = 2 * 128 * 64 * 2;  // A + B images
[[maybe_unused]] constexpr int RING_BYTES = NSTAGE * STAGE_BYTES;

// One operand image of one stage: 16 wave-instructions of 1 KB, 2 per wave (8 waves).
template <bool KSTRIDED>
TM_DEV void glds_tile(char* img, const bf16* X, int ld, int r0, int rmax, int k0, int wave, int lane) {
  typedef __attribute__((address_space(3))) void lds_t;
  typedef __attribute__((address_space(1))) void glb_t;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = wave * 2 + i;  // 1-KB piece of the image
    const bf16* src;
    if constexpr (!KSTRIDED) {   // rows r0.., 8 rows x 128 B per piece
      const int r = j * 8 + (lane >> 3), slot = lane & 7;
      const int c = slot ^ ((r >> 1) & 7);
      const int gr = min(r0 + r, rmax - 1);
      src = X + (size_t)gr * ld + k0 + c * 8;
    } else {                     // k-rows k0.., 4 rows x 256 B per piece
      const int k = j * 4 + (lane >> 4), slot = lane & 15;
      const int c = slot ^ (2 * (k & 3));
      const int gm = min(r0 + c * 8, rmax - 8);
      src = X + (size_t)(k0 + k) * ld + gm;
    }
    __builtin_amdgcn_global_load_lds((glb_t*)src, (lds_t*)(img + j * 1024), 16, 0, 0);
  }
}

// fragment of 32 rows (rb..rb+31) x 8 k (kb + 8h ..) from a k-contiguous image
TM_DEV bf16x8 frag_rows_sw(const char* img, int rb, int kb, int lane) {
  const int r = rb + (lane & 31), c = (kb >> 3) + (lane >> 5);
  return *(const bf16x8*)(img + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
}
// same fragment from a k-strided image via transposing reads
TM_DEV bf16x8 frag_kstr_sw(const char* img, int mb, int kb, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int m = mb + (g & 1) * 16 + 4 * p;
  const int k = kb + 8 * (g >> 1) + q;
  const int c = m >> 3, half = (m >> 2) & 1;
  typedef __attribute__((address_space(3))) bf16x4 lds_v4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_v4*)(img + k * 256 + ((c ^ (2 * (k & 3))) << 4) + half * 8));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_v4*)(img + (k + 4) * 256 + ((c ^ (2 * ((k + 4) & 3))) << 4) + half * 8));
  return (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int N>
TM_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// LDS fragment reads as inline asm: hipcc puts an `s_waitcnt vmcnt(0)` in front of every LDS
// read it cannot prove independent of an in-flight global_load_lds, which drains the prefetch
// ring at every k-step (the reason this ring lost to the register-staged loop in round 1).  The
// asm reads are ordered by explicit lgkmcnt waits + sched_barrier instead.
TM_DEV unsigned lds_u32(const void* p) { return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p; }
template <int OFF> TM_DEV void ds_b128(bf16x8& d, unsigned a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}
template <int OFF> TM_DEV void ds_tr64(bf16x4& d, unsigned a) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}
template <int N> TM_DEV void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
TM_DEV bf16x8 join4(const bf16x4& a, const bf16x4& b) { return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }

// lane addresses (relative to the operand image) of the 32-row x 8-k fragments of a 64-deep tile:
//   k-contiguous image (128 B rows, chunk c at slot c ^ ((r >> 1) & 7)): one address per k-step
//   k-strided image (256 B k-rows, chunk c at slot c ^ (2 (k & 3))): k-step s = +4096 s, the
//   second 4 k-rows +1024 (the swizzle depends on k & 3 only, fixed per lane)
TM_DEV void kc_addrs(unsigned (&a)[4], int rb, int lane) {
  const int r = rb + (lane & 31);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int c = 2 * s + (lane >> 5);
    a[s] = r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
  }
}
TM_DEV unsigned ks_addr(int mb, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int m = mb + (g & 1) * 16 + 4 * p;
  const int k = 8 * (g >> 1) + q;
  return k * 256 + (((m >> 3) ^ (2 * (k & 3))) << 4) + ((m >> 2) & 1) * 8;
}
template <bool KS, int S>
TM_DEV void rd_frag(bf16x8& f, unsigned base, const unsigned (&kc)[4]) {
  if constexpr (KS) {
    bf16x4 lo, hi;
    ds_tr64<S * 4096>(lo, base);
    ds_tr64<S * 4096 + 1024>(hi, base);
    f = join4(lo, hi);
  } else {
    ds_b128<0>(f, base + kc[S]);
  }
}

// one 64-deep k-tile of one wave's 32 x 64 subtile: 4 k-steps of 2 MFMAs, the LDS reads of
// step s+1 in flight while step s multiplies
// SWAP: the products are issued as (B, A) -- acc[j] holds the TRANSPOSED 32 x 32 tile (lane l:
// output row l & 31, 16 output columns per lane), the register layout gemm_pr_kernel stores from
template <bool A_KS, bool B_KS, bool SWAP = false>
TM_DEV void ring_tile_mma(f32x16 (&acc)[2], unsigned abase, unsigned b0, unsigned b1, const unsigned (&akc)[4],
                          const unsigned (&bkc0)[4], const unsigned (&bkc1)[4]) {
  constexpr int RS = (A_KS ? 2 : 1) + 2 * (B_KS ? 2 : 1);   // LDS reads per k-step
  auto mm = [](f32x16& c, const bf16x8& a, const bf16x8& b) {
    if constexpr (SWAP) mma16(c, b, a); else mma16(c, a, b);
  };
  bf16x8 a[2], b[2][2];
  rd_frag<A_KS, 0>(a[0], abase, akc); rd_frag<B_KS, 0>(b[0][0], b0, bkc0); rd_frag<B_KS, 0>(b[0][1], b1, bkc1);
  rd_frag<A_KS, 1>(a[1], abase, akc); rd_frag<B_KS, 1>(b[1][0], b0, bkc0); rd_frag<B_KS, 1>(b[1][1], b1, bkc1);
  wait_lgkm<RS>();
  mm(acc[0], a[0], b[0][0]);
  mm(acc[1], a[0], b[0][1]);
  rd_frag<A_KS, 2>(a[0], abase, akc); rd_frag<B_KS, 2>(b[0][0], b0, bkc0); rd_frag<B_KS, 2>(b[0][1], b1, bkc1);
  wait_lgkm<RS>();
  mm(acc[0], a[1], b[1][0]);
  mm(acc[1], a[1], b[1][1]);
  rd_frag<A_KS, 3>(a[1], abase, akc); rd_frag<B_KS, 3>(b[1][0], b0, bkc0); rd_frag<B_KS, 3>(b[1][1], b1, bkc1);
  wait_lgkm<RS>();
  mm(acc[0], a[0], b[0][0]);
  mm(acc[1], a[0], b[0][1]);
  wait_lgkm<0>();
  mm(acc[0], a[1], b[1][0]);
  mm(acc[1], a[1], b[1][1]);
}

// diagnostics (variant 8 only): per-workgroup shader-clock stamps of the ring kernel, read by
// tm_debug_gemm_stamps: [block][8] = realtime start, t start, first tile landed, k-loop done,
// accumulators staged, epilogue stores issued, stores retired, realtime end
__device__ unsigned long long g_gemm_stamps[2048 * 8];
template <bool ON>
TM_DEV void ring_stamp(unsigned long long (&ts)[8], int slot, bool real = false) {
  if constexpr (ON) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    if (real) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    else asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    ts[slot] = t;
  }
}

template <typename OutT, bool A_T, bool B_KN, int NS = NSTAGE, bool STAMP = false, int KIND = EK_ANY>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void gemm_ring_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                        OutT* __restrict__ C, tm_gemm_args g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ring_stamp<STAMP>(ts, 0, true);
  ring_stamp<STAMP>(ts, 1);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // 4 (M) x 2 (N) waves of 32 x 64
  int m0, n0, zs;
  tile_split_of_block(m0, n0, zs);
  const int kbeg = zs * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg) / 64 : 0;  // host guarantees 64 | (kend - kbeg)

  f32x16 acc[2];
  acc[0] = (f32x16){};
  acc[1] = (f32x16){};
  constexpr bool COLSUM = A_T && KIND == EK_SPLITK && !STAMP;
  const bool do_cs = COLSUM && g.colsum != nullptr && n0 == 0;   // block-uniform
  const int cs_c = tid & 15, cs_r = tid >> 4;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // fragment addresses relative to a stage: A at +0, B at +STAGE_BYTES/2
  unsigned akc[4] = {0, 0, 0, 0}, bkc0[4] = {0, 0, 0, 0}, bkc1[4] = {0, 0, 0, 0};
  unsigned aks = 0, bks0 = 0, bks1 = 0;
  if constexpr (A_T) aks = ks_addr(wm * 32, lane); else kc_addrs(akc, wm * 32, lane);
  if constexpr (B_KN) {
    bks0 = ks_addr(wn * 64, lane) + STAGE_BYTES / 2;
    bks1 = ks_addr(wn * 64 + 32, lane) + STAGE_BYTES / 2;
  } else {
    kc_addrs(bkc0, wn * 64, lane);
    kc_addrs(bkc1, wn * 64 + 32, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) { bkc0[s] += STAGE_BYTES / 2; bkc1[s] += STAGE_BYTES / 2; }
  }
  const unsigned ring = lds_u32(smem);

  auto issue = [&](int kt) {
    char* st = smem + (kt % NS) * STAGE_BYTES;
    const int k0 = kbeg + kt * 64;
    glds_tile<A_T>(st, A, g.lda, m0, g.M, k0, wave, lane);
    glds_tile<B_KN>(st + STAGE_BYTES / 2, B, g.ldb, n0, g.N, k0, wave, lane);
  };
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);

  for (int kt = 0; kt < nk; ++kt) {
    // this wave's pieces of tile kt have landed once at most (tiles issued after kt) x 4 loads remain
    const int ahead = min(NS - 2, nk - 1 - kt);
    if (ahead >= 2) wait_vm<8>(); else if (ahead == 1) wait_vm<4>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every wave's pieces landed; every wave done reading tile kt-1
    asm volatile("" ::: "memory");
    if (STAMP && kt == 0) ring_stamp<STAMP>(ts, 2);
    if (kt + NS - 1 < nk) issue(kt + NS - 1);  // overwrites tile kt-1's buffer
    const unsigned sb = ring + (kt % NS) * STAGE_BYTES;
    ring_tile_mma<A_T, B_KN>(acc, (A_T ? aks : 0) + sb, (B_KN ? bks0 : 0) + sb, (B_KN ? bks1 : 0) + sb,
                             akc, bkc0, bkc1);
    if constexpr (COLSUM) {
      // the bias gradient of the same dY: this tile's 64 k-rows of A summed per column (thread:
      // 16-B column chunk cs_c of k-rows cs_r and cs_r + 32), behind the tile's MFMAs
      if (do_cs) {
        const char* img = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int kk = cs_r + 32 * j;
          const bf16x8 v = *(const bf16x8*)(img + kk * 256 + ((cs_c ^ (2 * (kk & 3))) << 4));
#pragma unroll
          for (int e = 0; e < 8; ++e) csum[e] += (float)v[e];
        }
      }
    }
  }
  ring_stamp<STAMP>(ts, 3);
  __syncthreads();  // all fragment reads done before the epilogue reuses the ring
  float* ep = (float*)smem;
#pragma unroll
  for (int j = 0; j < 2; ++j) stage_acc(ep, acc[j], wm * 32, wn * 64 + j * 32, lane);
  __syncthreads();
  ring_stamp<STAMP>(ts, 4);
  if (STAMP && g.drop_scale < 0.f) {
    // diagnostics: image reads only, no global stores (drop_scale -1) or plain bf16/f32 stores of
    // the image with no other epilogue work (drop_scale -2)
    const float* ep2 = (const float*)smem;
    for (int c = tid; c < BM * 16; c += 512) {
      const int lr = c / 16, lc = (c % 16) * 8;
      const f32x4 lo = *(const f32x4*)(ep2 + lr * EP_ROW + lc), hi = *(const f32x4*)(ep2 + lr * EP_ROW + lc + 4);
      if (g.drop_scale < -1.5f) {
        OutT* dst = C + (size_t)(m0 + lr) * g.ldc + n0 + lc;
        if (m0 + lr < g.M) {
          vec8<OutT> o;
          for (int e = 0; e < 4; ++e) { o[e] = from_f<OutT>(lo[e]); o[e + 4] = from_f<OutT>(hi[e]); }
          store8<OutT>(dst, o);
        }
      } else {
        asm volatile("" ::"v"(lo), "v"(hi));
      }
    }
  } else
  gemm_epilogue_rows<OutT, BN, BM, 512, KIND>(smem, C, g, m0, n0, zs);
  if constexpr (COLSUM) {
    if (do_cs) {
      // the 32 k-row groups of each column chunk: lanes c, c + 16, c + 32, c + 48 of a wave, then
      // the 8 waves through LDS (the epilogue is done with it), summed in wave order
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        csum[e] += __shfl_xor(csum[e], 16, 64);
        csum[e] += __shfl_xor(csum[e], 32, 64);
      }
      __syncthreads();
      float* red = (float*)smem;   // [8 waves][128 columns]
      if (lane < 16) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red[wave * 128 + cs_c * 8 + e] = csum[e];
      }
      __syncthreads();
      if (tid < 128 && m0 + tid < g.M) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) s += red[w * 128 + tid];
        g.colsum[(size_t)zs * g.M + m0 + tid] = s;
      }
    }
  }
  if constexpr (STAMP) {
    ring_stamp<STAMP>(ts, 5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ring_stamp<STAMP>(ts, 6);
    ring_stamp<STAMP>(ts, 7, true);
    const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;   // split-K grids too
    if (tid < 8 && blk < 2048) {
      unsigned long long v = ts[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) v = tid == i ? ts[i] : v;
      g_gemm_stamps[blk * 8 + tid] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// 160 x 128 tiles for the M = n' = 8448-row GEMMs of the step (k-contiguous A only).  At 8448 rows
// a 128-row tiling is 66 row tiles: 264 tiles for N = 512 (8 more than 256 CUs: eight CUs take two
// tiles and set the launch time) and 792 for N = 1536 (3.1 per CU); 160 rows give 53 row tiles:
// 212 tiles (one round) and 636.  10 waves = 5 (M) x 2 (N) of the ring kernel's 32 x 64 subtiles,
// the same 2-stage LDS-DMA ring (A 20 KB + B 16 KB per stage: 72 KB, two workgroups per CU), the
// same fragment reads; the epilogue stages the tile in three row passes (64, 64, 32 rows) through
// the ring memory.
constexpr int BM160 = 160;
constexpr int R160_A = BM160 * 128, R160_STAGE = R160_A + 128 * 128;   // bytes: A image, A + B image

// XCD-contiguous renumbering as tile_split_of_block, 160-row tiles, no split
TM_DEV void tile160_of_block(int& m0, int& n0) {
  const int ntx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int orig = blockIdx.y * ntx + blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  m0 = (id / ntx) * BM160;
  n0 = (id % ntx) * BN;
}

template <typename OutT, bool B_KN, int KIND = EK_ANY>
__global__ __launch_bounds__(640) void gemm_ring160_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           OutT* __restrict__ C, tm_gemm_args g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) void lds_t;
  typedef __attribute__((address_space(1))) void glb_t;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;   // 5 (M) x 2 (N) waves of 32 x 64
  int m0, n0;
  tile160_of_block(m0, n0);
  const int nk = g.K / 64;                   // host guarantees 64 | K

  f32x16 acc[2];
  acc[0] = (f32x16){};
  acc[1] = (f32x16){};
  unsigned akc[4], bkc0[4] = {0, 0, 0, 0}, bkc1[4] = {0, 0, 0, 0};
  unsigned bks0 = 0, bks1 = 0;
  kc_addrs(akc, wm * 32, lane);
  if constexpr (B_KN) {
    bks0 = ks_addr(wn * 64, lane) + R160_A;
    bks1 = ks_addr(wn * 64 + 32, lane) + R160_A;
  } else {
    kc_addrs(bkc0, wn * 64, lane);
    kc_addrs(bkc1, wn * 64 + 32, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) { bkc0[s] += R160_A; bkc1[s] += R160_A; }
  }
  const unsigned ring = lds_u32(smem);
  // DMA pieces (1 KB wave-instructions): A = 20 (wave w: 2w, 2w + 1), B = 16 (waves 0-7: 2w, 2w + 1)
  auto issue = [&](int kt) {
    char* st = smem + (kt & 1) * R160_STAGE;
    const int k0 = kt * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = wave * 2 + i;
      const int r = j * 8 + (lane >> 3), slot = lane & 7;
      const int c = slot ^ ((r >> 1) & 7);
      const int gr = min(m0 + r, g.M - 1);
      __builtin_amdgcn_global_load_lds((glb_t*)(A + (size_t)gr * g.lda + k0 + c * 8), (lds_t*)(st + j * 1024), 16, 0, 0);
    }
    if (wave < 8) glds_tile<B_KN>(st + R160_A, B, g.ldb, n0, g.N, k0, wave, lane);
  };
  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's pieces of tile kt landed (tile kt + 1 not yet issued: wait for all)
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();   // every wave's pieces landed; every wave done reading tile kt - 1
    asm volatile("" ::: "memory");
    if (kt + 1 < nk) issue(kt + 1);  // overwrites tile kt - 1's buffer
    const unsigned sb = ring + (kt & 1) * R160_STAGE;
    ring_tile_mma<false, B_KN>(acc, sb, (B_KN ? bks0 : 0) + sb, (B_KN ? bks1 : 0) + sb, akc, bkc0, bkc1);
  }
  __syncthreads();   // all fragment reads done before the epilogue reuses the ring
  float* ep = (float*)smem;
  // three row passes: waves rows [0, 64), [64, 128), [128, 160)
#pragma unroll 1
  for (int pass = 0; pass < 3; ++pass) {
    const int rlo = pass * 64, rows = pass < 2 ? 64 : 32;
    if (wm * 32 >= rlo && wm * 32 < rlo + rows) {
#pragma unroll
      for (int j = 0; j < 2; ++j) stage_acc(ep, acc[j], wm * 32 - rlo, wn * 64 + j * 32, lane);
    }
    __syncthreads();
    if (tid < 512) {
      if (rows == 64) gemm_epilogue_rows<OutT, BN, 64, 512, KIND>(smem, C, g, m0 + rlo, n0, 0);
      else gemm_epilogue_rows<OutT, BN, 32, 512, KIND>(smem, C, g, m0 + rlo, n0, 0);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Persistent bf16 GEMM: one 512-thread workgroup per CU walks its tiles (t = blockIdx.x +
// i * gridDim.x, XCD-clustered) as ONE stream of 64-deep k-steps, so the global_load_lds ring
// keeps prefetching across tile boundaries: the next tile's first k-tiles are in flight while
// the current tile's epilogue runs (from its own LDS region).  Ring: 3 stages x 32 KB; epilogue
// image 64 rows x EP_ROW fp32 (two halves per tile).  Same fragment reads and epilogue as the
// ring kernel above; the split-K index rides in the tile id.
constexpr int PSTAGE = 3;
[[maybe_unused]] constexpr int PERSIST_LDS = PSTAGE * STAGE_BYTES + 64 * EP_ROW * 4;

struct PTile {
  int i, t, m0, n0, split, kbeg, nk, kt;
};

TM_DEV void ptile_set(PTile& c, int ntiles, int tiles_m, int tiles_n, const tm_gemm_args& g) {
  c.t = blockIdx.x + c.i * gridDim.x;
  c.kt = 0;
  if (c.t >= ntiles) { c.nk = 0; return; }
  // XCD clustering: workgroup b runs on XCD b % 8 and owns tiles t = b (mod gridDim.x); renumber
  // so each XCD's tiles form contiguous row-major runs (shared A panels stay in its L2)
  const int per = tiles_m * tiles_n;
  const int x = c.t % 8, q = ntiles / 8, r = ntiles % 8;
  const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + c.t / 8;
  c.split = id / per;
  const int rr = id % per;
  c.m0 = (rr / tiles_n) * BM;
  c.n0 = (rr % tiles_n) * BN;
  c.kbeg = c.split * g.k_per_split;
  c.nk = (min(g.K, c.kbeg + g.k_per_split) - c.kbeg) / 64;
}

template <typename OutT, bool A_T, bool B_KN>
__global__ __launch_bounds__(512) void gemm_persist_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           OutT* __restrict__ C, tm_gemm_args g, int tiles_m,
                                                           int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* epi = smem + PSTAGE * STAGE_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = tiles_m * tiles_n * g.splits;

  unsigned akc[4] = {0, 0, 0, 0}, bkc0[4] = {0, 0, 0, 0}, bkc1[4] = {0, 0, 0, 0};
  unsigned aks = 0, bks0 = 0, bks1 = 0;
  if constexpr (A_T) aks = ks_addr(wm * 32, lane); else kc_addrs(akc, wm * 32, lane);
  if constexpr (B_KN) {
    bks0 = ks_addr(wn * 64, lane) + STAGE_BYTES / 2;
    bks1 = ks_addr(wn * 64 + 32, lane) + STAGE_BYTES / 2;
  } else {
    kc_addrs(bkc0, wn * 64, lane);
    kc_addrs(bkc1, wn * 64 + 32, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) { bkc0[s] += STAGE_BYTES / 2; bkc1[s] += STAGE_BYTES / 2; }
  }
  const unsigned ring = lds_u32(smem);

  PTile is{}, cs{};
  is.i = 0;
  ptile_set(is, ntiles, tiles_m, tiles_n, g);
  while (is.nk == 0 && is.t < ntiles) { ++is.i; ptile_set(is, ntiles, tiles_m, tiles_n, g); }  // empty splits
  cs = is;
  int issued = 0, done = 0;
  auto issue = [&]() {
    char* st = smem + (issued % PSTAGE) * STAGE_BYTES;
    const int k0 = is.kbeg + is.kt * 64;
    glds_tile<A_T>(st, A, g.lda, is.m0, g.M, k0, wave, lane);
    glds_tile<B_KN>(st + STAGE_BYTES / 2, B, g.ldb, is.n0, g.N, k0, wave, lane);
    ++issued;
    if (++is.kt == is.nk) {
      do { ++is.i; ptile_set(is, ntiles, tiles_m, tiles_n, g); } while (is.nk == 0 && is.t < ntiles);
    }
  };
#pragma unroll
  for (int p = 0; p < PSTAGE - 1; ++p)
    if (is.t < ntiles) issue();

  f32x16 acc[2];
  acc[0] = (f32x16){};
  acc[1] = (f32x16){};
  while (cs.t < ntiles) {
    // step `done` landed once at most (issued - done - 1) younger steps (4 loads each) remain
    if (issued - done - 1 >= 1) wait_vm<4>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every wave's pieces landed; every wave done with step done-1
    asm volatile("" ::: "memory");
    if (is.t < ntiles) issue();    // overwrites step done-1's slot
    const unsigned sb = ring + (done % PSTAGE) * STAGE_BYTES;
    ring_tile_mma<A_T, B_KN>(acc, (A_T ? aks : 0) + sb, (B_KN ? bks0 : 0) + sb, (B_KN ? bks1 : 0) + sb,
                             akc, bkc0, bkc1);
    ++done;
    if (++cs.kt == cs.nk) {
      // epilogue of this tile from the epilogue image (two 64-row halves); the next tile's
      // first k-steps are already in flight
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        if ((wm >> 1) == half) {
#pragma unroll
          for (int j = 0; j < 2; ++j) stage_acc((float*)epi, acc[j], (wm & 1) * 32, wn * 64 + j * 32, lane);
        }
        __syncthreads();
        gemm_epilogue_rows<OutT, BN, 64, 512>(epi, C, g, cs.m0 + half * 64, cs.n0, cs.split);
        __syncthreads();
      }
      wait_vm<0>();   // the epilogue's own loads / stores (their count is data dependent)
      acc[0] = (f32x16){};
      acc[1] = (f32x16){};
      do { ++cs.i; ptile_set(cs, ntiles, tiles_m, tiles_n, g); } while (cs.nk == 0 && cs.t < ntiles);
    }
  }
}

#ifdef TM_DIAG
// ---------------------------------------------------------------------------
// Persistent ring GEMM with the epilogue straight from the accumulator registers (gemm_pr_kernel):
// two 512-thread workgroups per CU (64 KB of LDS each: the 2-stage LDS-DMA ring and nothing else),
// each walking its tiles t = blockIdx.x + i * gridDim.x (XCD-clustered, ptile_set) as ONE stream of
// 64-deep k-steps.  What it removes, per tile, from the ring kernel's timeline (stamps,
// scripts/dev/gemm_stamps2.py, profiles/r05c_gemm_stamps.txt -- QKV: first tile landed 2.8 k,
// k-loop 10.6 k, accumulator staging 1.2 k, epilogue 2.6 k cycles per tile):
//   * the first k-step of the next tile is already in flight while this tile's epilogue runs;
//   * no LDS epilogue image: the products are issued transposed (ring_tile_mma<.., SWAP>), so each
//     lane holds 16 output COLUMNS of one output row; one cross-half exchange (lanes l, l ^ 32)
//     gives every lane 8 consecutive columns -> the epilogue works on 8-column row chunks as the
//     staged one does (bias, pre-activation, GELU, dropout, residual, row map, QKV scatter) and
//     stores 16 B (bf16) / 32 B (fp32) per lane with no barrier and no LDS round trip;
//   * the two workgroups of a CU drift apart after their first tiles, so one's epilogue and first
//     operand fill overlap the other's MFMA k-loop.
// Chunk (j, p) of a lane: row m0 + 32 wm + (l & 31), columns n0 + 64 wn + 32 j + 16 p + 8 (l >> 5).
constexpr int PR_NS = 2;
[[maybe_unused]] constexpr int PR_LDS = PR_NS * STAGE_BYTES;   // 64 KB

template <typename OutT, int KIND>
TM_DEV void pr_epilogue_chunk(OutT* __restrict__ C, const tm_gemm_args& g, int m, int n, const float (&v)[8],
                              uint64_t seed) {
  const int ne = min(8, g.N - n);
  if (ne <= 0 || m >= g.M) return;
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g.bias) {
    if (ne == 8 && ((uintptr_t)g.bias & 15) == 0) { const f32x8 t8 = load8<float>(g.bias + n); for (int e = 0; e < 8; ++e) bv[e] = t8[e]; }
    else { for (int e = 0; e < ne; ++e) bv[e] = g.bias[n + e]; }
  }
  if constexpr (KIND == EK_QKV) {   // 8 columns never straddle a head (dh % 8 == 0, checked on the host)
    const int inner = g.nh * g.dh;
    const int which = n / inner, hh = (n % inner) / g.dh, d = n % g.dh;
    const float qs = which == 0 ? g.qscale : 1.f;
    const int bag = m / g.seq, t = m - bag * g.seq;
    OutT* dst = C + ((((long long)which * g.nbags + bag) * g.nh + hh) * g.seq + t) * g.dh + d;
    vec8<OutT> o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f<OutT>((v[e] * g.alpha + bv[e]) * qs);
    store8<OutT>(dst, o);
    return;
  } else if constexpr (KIND == EK_PLAIN) {
    vec8<OutT> o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f<OutT>(v[e] * g.alpha + bv[e]);
    OutT* dst = C + (size_t)m * g.ldc + n;
    if (ne == 8 && g.ldc % 8 == 0) store8<OutT>(dst, o);
    else { for (int e = 0; e < ne; ++e) dst[e] = o[e]; }
    return;
  } else {
    // runtime mode: row map (TransMIL grid duplication / padding skip), pre-activation, GELU,
    // dropout, residual / accumulate -- the same per-element order as gemm_epilogue_rows
    int row = m, dup = -1;
    if (g.grp_in > 0) {
      const int bag = m / g.grp_in, t = m - bag * g.grp_in - g.skip;
      if (t < 0) return;
      if (t < g.dup_n) dup = bag * g.grp_out + g.dup_off + t;
      row = bag * g.grp_out + g.out_off + t;
    }
    const bool vec = ne == 8 && g.ldc % 8 == 0 && (!g.pre || g.ld_pre % 8 == 0);
    const size_t off = (size_t)row * g.ldc + n;
    float addr[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, addc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (g.resid) {
      if (vec) { const f32x8 t8 = load8<float>(g.resid + off); for (int e = 0; e < 8; ++e) addr[e] = t8[e]; }
      else { for (int e = 0; e < ne; ++e) addr[e] = g.resid[off + e]; }
    }
    if (g.accumulate) {
      if (vec) { const vec8<OutT> t8 = load8<OutT>(C + off); for (int e = 0; e < 8; ++e) addc[e] = to_f(t8[e]); }
      else { for (int e = 0; e < ne; ++e) addc[e] = to_f(C[off + e]); }
    }
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = v[e] * g.alpha + bv[e];
    vec8<OutT> pre8, out8;
    if (g.pre) {
#pragma unroll
      for (int e = 0; e < 8; ++e) pre8[e] = from_f<OutT>(x[e]);
    }
    if (g.gelu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = gelu_erf(x[e]);
    }
    if (g.drop_p > 0.f) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float u = dropout_u01(seed, (uint32_t)row, (uint32_t)(n + e));
        x[e] = (u >= g.drop_p) ? x[e] * g.drop_scale : 0.f;
      }
    }
    // as gemm_epilogue_rows: + residual, then + the stored C (accumulate), in that order
    if (g.resid) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] += addr[e];
    }
    if (g.accumulate) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] += addc[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) out8[e] = from_f<OutT>(x[e]);
    if (vec) {
      if (g.pre) store8<OutT>((OutT*)g.pre + (size_t)m * g.ld_pre + n, pre8);
      store8<OutT>(C + off, out8);
      if (dup >= 0) store8<OutT>(C + (size_t)dup * g.ldc + n, out8);
    } else {
      for (int e = 0; e < ne; ++e) {
        if (g.pre) ((OutT*)g.pre)[(size_t)m * g.ld_pre + n + e] = pre8[e];
        C[off + e] = out8[e];
        if (dup >= 0) C[(size_t)dup * g.ldc + n + e] = out8[e];
      }
    }
  }
}

template <typename OutT, bool B_KN, int KIND>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void gemm_pr_kernel(
    const bf16* __restrict__ A, const bf16* __restrict__ B, OutT* __restrict__ C, tm_gemm_args g, int tiles_m,
    int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;   // 4 (M) x 2 (N) waves of 32 x 64
  const int ntiles = tiles_m * tiles_n;       // splits == 1 (host-checked)

  unsigned akc[4], bkc0[4] = {0, 0, 0, 0}, bkc1[4] = {0, 0, 0, 0};
  unsigned bks0 = 0, bks1 = 0;
  kc_addrs(akc, wm * 32, lane);
  if constexpr (B_KN) {
    bks0 = ks_addr(wn * 64, lane) + STAGE_BYTES / 2;
    bks1 = ks_addr(wn * 64 + 32, lane) + STAGE_BYTES / 2;
  } else {
    kc_addrs(bkc0, wn * 64, lane);
    kc_addrs(bkc1, wn * 64 + 32, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) { bkc0[s] += STAGE_BYTES / 2; bkc1[s] += STAGE_BYTES / 2; }
  }
  const unsigned ring = lds_u32(smem);
  const uint64_t seed = (KIND == EK_ANY && g.drop_p > 0.f) ? effective_seed(g.seed, g.seed_ptr) : 0;

  PTile is{}, cs{};
  is.i = 0;
  ptile_set(is, ntiles, tiles_m, tiles_n, g);
  cs = is;
  int issued = 0, done = 0;
  auto issue = [&]() {
    char* st = smem + (issued % PR_NS) * STAGE_BYTES;
    const int k0 = is.kt * 64;
    glds_tile<false>(st, A, g.lda, is.m0, g.M, k0, wave, lane);
    glds_tile<B_KN>(st + STAGE_BYTES / 2, B, g.ldb, is.n0, g.N, k0, wave, lane);
    ++issued;
    if (++is.kt == is.nk) { ++is.i; ptile_set(is, ntiles, tiles_m, tiles_n, g); }
  };
  if (is.t < ntiles) issue();

  f32x16 acc[2];
  acc[0] = (f32x16){};
  acc[1] = (f32x16){};
  const int h = lane >> 5, r32 = lane & 31;
  while (cs.t < ntiles) {
    // step `done` landed once at most (issued - done - 1) younger steps (4 loads each) remain; after
    // an epilogue none is younger, and the wait also retires that epilogue's stores
    if (issued - done - 1 >= 1) wait_vm<4>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every wave's pieces landed; every wave done with step done-1
    asm volatile("" ::: "memory");
    if (is.t < ntiles) issue();    // overwrites step done-1's slot (possibly the next tile's first step)
    const unsigned sb = ring + (done % PR_NS) * STAGE_BYTES;
    ring_tile_mma<false, B_KN, true>(acc, sb, (B_KN ? bks0 : 0) + sb, (B_KN ? bks1 : 0) + sb, akc, bkc0, bkc1);
    ++done;
    if (++cs.kt == cs.nk) {
      // epilogue from registers: acc[j] lane l = row 32 wm + r32 (of the tile), columns
      // 64 wn + 32 j + acc_row(i, h); the (l, l ^ 32) exchange gives 8 consecutive columns
      const int m = cs.m0 + wm * 32 + r32;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int q0 = 2 * p, q1 = 2 * p + 1;
          float send[4], recv[4], v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) send[e] = h ? acc[j][4 * q0 + e] : acc[j][4 * q1 + e];
#pragma unroll
          for (int e = 0; e < 4; ++e) recv[e] = __shfl_xor(send[e], 32, 64);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = h ? recv[e] : acc[j][4 * q0 + e];
            v[4 + e] = h ? acc[j][4 * q1 + e] : recv[e];
          }
          pr_epilogue_chunk<OutT, KIND>(C, g, m, cs.n0 + wn * 64 + j * 32 + 16 * p + 8 * h, v, seed);
        }
      }
      acc[0] = (f32x16){};
      acc[1] = (f32x16){};
      ++cs.i;
      ptile_set(cs, ntiles, tiles_m, tiles_n, g);
    }
  }
}
#endif  // TM_DIAG (gemm_pr_kernel: measured slower on every step shape, profiles/r05d_ab_gemm_pr_rejected.txt)

// ---------------------------------------------------------------------------
// Big-tile bf16 GEMM: 256 x TBN (256 or 128) per 512-thread workgroup.  A 128 x 128 tile moves
// 32 KB of operands per 64-deep k-step for 2 MFLOP (64 flop/B): at 2.5 PF that needs ~39 TB/s of
// L2 -> CU operand bandwidth, which the chip does not have (the 128-tile kernels above run at
// 15 % of the MFMA peak).  256 x 256 halves the bytes per flop (128 flop/B); 256 x 128 serves
// the N = 512 shapes with twice the workgroups.  8 waves: 2 (M) x 4 (N) of 128 x 64 (TBN 256)
// or 4 x 2 of 64 x 64 (TBN 128); operands by global_load_lds into a 2- / 3-stage ring of
// swizzled images (k-contiguous: 128-B rows; k-strided: 64 k-rows of 2 x TBM / TBN bytes), LDS
// fragment reads as inline asm (no vmcnt(0) drains), epilogue staged 64 rows at a time.
constexpr int GBM = 256;

template <int ROWS>
TM_DEV void glds_big(char* img, const bf16* X, int ld, int r0, int rmax, int k0, bool kstr, int wave, int lane) {
  typedef __attribute__((address_space(3))) void lds_t;
  typedef __attribute__((address_space(1))) void glb_t;
  constexpr int PIECES = ROWS * 128 / 1024;          // 1-KB pieces per image (32 or 16)
  constexpr int PPW = PIECES / 8;                    // per wave
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int j = wave * PPW + i;
    const bf16* src;
    if (!kstr) {                 // 8 rows x 128 B per piece, chunk c of row r at slot c ^ ((r >> 1) & 7)
      const int r = j * 8 + (lane >> 3), slot = lane & 7;
      const int c = slot ^ ((r >> 1) & 7);
      const int gr = min(r0 + r, rmax - 1);
      src = X + (size_t)gr * ld + k0 + c * 8;
    } else {                     // k-rows of ROWS*2 bytes: 1024 / (ROWS*2) k-rows per piece
      constexpr int CH = ROWS / 8;                     // 16-B chunks per k-row (32 or 16)
      constexpr int KPP = 64 / CH;                     // k-rows per piece (2 or 4)
      const int k = j * KPP + lane / CH, slot = lane % CH;
      const int c = slot ^ (2 * (k & 3));
      const int gm = min(r0 + c * 8, rmax - 8);
      src = X + (size_t)(k0 + k) * ld + gm;
    }
    __builtin_amdgcn_global_load_lds((glb_t*)src, (lds_t*)(img + j * 1024), 16, 0, 0);
  }
}

// k-strided image lane address (k-step 0, first 4 k-rows) for a 32-wide fragment at mb
template <int ROWS>
TM_DEV unsigned ks_addr_big(int mb, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int m = mb + (g & 1) * 16 + 4 * p;
  const int k = 8 * (g >> 1) + q;
  return k * (ROWS * 2) + (((m >> 3) ^ (2 * (k & 3))) << 4) + ((m >> 2) & 1) * 8;
}

template <bool KS, int ROWS, int S>
TM_DEV void rd_big(bf16x8& f, unsigned base, unsigned kc_s) {
  if constexpr (KS) {
    bf16x4 lo, hi;
    ds_tr64<S * 16 * ROWS * 2>(lo, base);
    ds_tr64<S * 16 * ROWS * 2 + 4 * ROWS * 2>(hi, base);
    f = join4(lo, hi);
  } else {
    ds_b128<0>(f, base + kc_s);
  }
}

constexpr int BIG_EROWS = 128;   // rows per epilogue pass of the big-tile kernel
template <typename OutT, bool A_T, bool B_KN, int TBN, bool STAMP = false>   // STAMP: diagnostic variant 12
__global__ __launch_bounds__(512) void gemm_big_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                       OutT* __restrict__ C, tm_gemm_args g) {
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ring_stamp<STAMP>(ts, 0, true);
  ring_stamp<STAMP>(ts, 1);
  constexpr int WM = TBN == 256 ? 2 : 4, WN = 8 / WM;
  constexpr int FM = GBM / WM / 32, FN = TBN / WN / 32;      // 32x32 MFMA tiles per wave
  constexpr int A_BYTES = GBM * 128, B_BYTES = TBN * 128, STG = A_BYTES + B_BYTES;
  constexpr int NS = TBN == 256 ? 2 : 3;
  constexpr int RS = FM * (A_T ? 2 : 1) + FN * (B_KN ? 2 : 1);   // LDS reads per k-step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware tile order (as tile_of_block, 256 x TBN tiles)
  int m0, n0;
  {
    const int ntx = gridDim.x, nwg = gridDim.x * gridDim.y;
    const int orig = blockIdx.y * ntx + blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
    m0 = (id / ntx) * GBM;
    n0 = (id % ntx) * TBN;
  }
  const int kbeg = blockIdx.z * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg) / 64 : 0;

  // per-lane fragment addresses relative to a stage
  unsigned ab[FM], bb[FN];
  unsigned akc[FM][4], bkc[FN][4];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int rb = wm * (GBM / WM) + i * 32;
    if constexpr (A_T) ab[i] = ks_addr_big<GBM>(rb, lane);
    else { ab[i] = 0; kc_addrs(akc[i], rb, lane); }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int cb = wn * (TBN / WN) + j * 32;
    if constexpr (B_KN) bb[j] = ks_addr_big<TBN>(cb, lane) + A_BYTES;
    else {
      bb[j] = A_BYTES;
      kc_addrs(bkc[j], cb, lane);
    }
  }
  const unsigned ring = lds_u32(smem);
  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x16){};

  auto issue = [&](int kt) {
    char* st = smem + (kt % NS) * STG;
    const int k0 = kbeg + kt * 64;
    glds_big<GBM>(st, A, g.lda, m0, g.M, k0, A_T, wave, lane);
    glds_big<TBN>(st + A_BYTES, B, g.ldb, n0, g.N, k0, B_KN, wave, lane);
  };
  constexpr int LPW = (GBM + TBN) * 128 / 1024 / 8;       // loads per wave per stage
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);

  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NS - 2, nk - 1 - kt);
    if (ahead >= 1) wait_vm<LPW>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (STAMP && kt == 0) ring_stamp<STAMP>(ts, 2);
    if (kt + NS - 1 < nk) issue(kt + NS - 1);
    const unsigned sb = ring + (kt % NS) * STG;
    bf16x8 af[2][FM], bf[2][FN];
#define TM_BIG_READ(BUF, S)                                                                       \
    _Pragma("unroll") for (int i = 0; i < FM; ++i) rd_big<A_T, GBM, S>(af[BUF][i], ab[i] + sb, A_T ? 0u : akc[i][S]); \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) rd_big<B_KN, TBN, S>(bf[BUF][j], bb[j] + sb, B_KN ? 0u : bkc[j][S]);
#define TM_BIG_MMA(BUF)                                                                           \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                \
      _Pragma("unroll") for (int j = 0; j < FN; ++j) mma16(acc[i][j], af[BUF][i], bf[BUF][j]);
    TM_BIG_READ(0, 0)
    TM_BIG_READ(1, 1)
    wait_lgkm<RS>();
    TM_BIG_MMA(0)
    TM_BIG_READ(0, 2)
    wait_lgkm<RS>();
    TM_BIG_MMA(1)
    TM_BIG_READ(1, 3)
    wait_lgkm<RS>();
    TM_BIG_MMA(0)
    wait_lgkm<0>();
    TM_BIG_MMA(1)
#undef TM_BIG_READ
#undef TM_BIG_MMA
  }
  ring_stamp<STAMP>(ts, 3);
  __syncthreads();   // every fragment read done: the ring becomes the epilogue image
  ring_stamp<STAMP>(ts, 4);
  float* ep = (float*)smem;
  constexpr int ROWF = TBN + 8;
  // two passes of BIG_EROWS = 128 rows (the fp32 image, 135 KB at TBN = 256, fits beside nothing
  // else; four 64-row passes took 17.6 k cycles of a 45 k-cycle workgroup: twice the barriers and
  // staging phases, scripts/dev/qkv_big_stamps.py)
#pragma unroll
  for (int ph = 0; ph < GBM / BIG_EROWS; ++ph) {
    // rows BIG_EROWS ph ..: wave row wm covers rows wm * GBM/WM .. ; its frags i with 32-row blocks inside
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rb = wm * (GBM / WM) + i * 32;
      if (rb / BIG_EROWS == ph) {
        const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int cb = wn * (TBN / WN) + j * 32;
#pragma unroll
          for (int r = 0; r < 16; ++r) ep[(rb - BIG_EROWS * ph + acc_row(r, h)) * ROWF + cb + l32] = acc[i][j][r];
        }
      }
    }
    __syncthreads();
    gemm_epilogue_rows<OutT, TBN, BIG_EROWS, 512>((char*)smem, C, g, m0 + ph * BIG_EROWS, n0);
    __syncthreads();
  }
  if constexpr (STAMP) {   // (slots as the ring kernel's; 4 = staged is the k-loop barrier here)
    ring_stamp<STAMP>(ts, 5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ring_stamp<STAMP>(ts, 6);
    ring_stamp<STAMP>(ts, 7, true);
    const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (tid < 8 && blk < 2048) {
      unsigned long long v = ts[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) v = tid == i ? ts[i] : v;
      g_gemm_stamps[blk * 8 + tid] = v;
    }
  }
}

template <typename OutT, int TBN>
constexpr int big_lds() {
  constexpr int ring = (TBN == 256 ? 2 : 3) * (GBM + TBN) * 128;
  constexpr int epi = BIG_EROWS * (TBN + 8) * 4;
  static_assert(epi <= 160 * 1024, "big-tile epilogue image exceeds the LDS");
  return ring > epi ? ring : epi;
}

template <typename T, bool A_T, bool B_KN, int NBUF = 2>
constexpr size_t gemm_smem() {
  constexpr size_t main = NBUF * (tile_elems<T, A_T>() + tile_elems<T, B_KN>()) * sizeof(T);
  constexpr size_t epi = (size_t)(BM / 2) * EP_ROW * sizeof(float);
  return main > epi ? main : epi;
}

// 0 = the 2-stage 128 x 128 DMA ring where it applies (bf16, 64 | K per split), else the
// register-staged loop with 1 LDS buffer; 1 = register-staged, 2 LDS buffers; 2 = 4-stage ring;
// 3 = register-staged, 1 LDS buffer; 4 = persistent 128 x 128 DMA ring; 5 = 2-stage ring; 6 =
// 3-stage ring; 7 = 256 x 256 / 256 x 128 big-tile kernel.  The 2-stage ring (69.6 KB of LDS with
// its epilogue image) keeps two workgroups per CU, which is what wins on these shapes: at
// M = 8448 rows 264 tiles of 128 x 128 are a 256-CU wave plus 8 tiles, and the second workgroup
// on a CU shares its operand intake instead of waiting for a second round (QKV 32.2 vs 36.5 us
// big-tile; to_out 17.9 vs 21.0 register-staged; dxn 31.1 vs 36.4; fc1 18.3 vs 25.3; weight
// grads 19.3 / 35.6 / 29.1 vs 21.5 / 39.1 / 38.1; scripts/dev/gemm_shapes.py)
#ifdef TM_DIAG
int g_gemm_variant = 0;
#endif
#define GEMM_VARIANT TM_DIAG_VAR(g_gemm_variant)

// the specialised epilogue a launch can use (EK_ANY keeps the runtime-mode one)
inline int epilogue_kind(const tm_gemm_args& g) {
  if (g.mode == TM_EPI_SPLITK) return EK_SPLITK;
  if (g.mode == TM_EPI_QKV) return EK_QKV;
  if (!g.pre && !g.gelu && g.drop_p <= 0.f && !g.resid && !g.accumulate && g.grp_in <= 0) return EK_PLAIN;
  return EK_ANY;
}

template <typename OutT>
bool ring_ok(const tm_gemm_args& g) {
  if (GEMM_VARIANT != 0 && GEMM_VARIANT != 8 && GEMM_VARIANT != 9 && (GEMM_VARIANT < 2 || GEMM_VARIANT > 6 || GEMM_VARIANT == 3)) return false;
  // whole 64-deep k-tiles in every split; k-strided operands need >= 8 rows/cols (clamped 16-B pieces)
  if (g.K % 64 != 0 || (g.splits > 1 && g.k_per_split % 64 != 0)) return false;
  if ((g.a_trans && g.M < 8) || (g.b_kn && g.N < 8)) return false;
  if (g.a_trans && g.M % 8 != 0) return false;
  if (g.b_kn && g.N % 8 != 0) return false;
  return true;
}

// 160-row tiles (k-contiguous A, no split)
// (diagnostic build: variant 9 never, 10 wherever valid)
inline bool use_ring160(const tm_gemm_args& g) {
  if (g.a_trans || g.splits != 1 || g.K % 64 != 0 || g.M < BM160 || g.mode == TM_EPI_SPLITK) return false;
  if (g.b_kn && (g.N % 8 != 0 || g.N < 8)) return false;
  if (GEMM_VARIANT == 10) return true;
  if (GEMM_VARIANT != 0) return false;
  // the heavy runtime-mode epilogue (dropout hash, residual, row map: to_out) stays on 128-row
  // tiles: in the step it ran 22.6 vs 20 us there (three staging passes of 512 of 640 threads)
  if (epilogue_kind(g) == EK_ANY) return false;
  // where 128-row tiles spill past one per CU and 160-row tiles do not (N = 512 at 8448 rows: dxn
  // 28.8 -> 22.9 us, to_out 16.2 -> 13.9, dmerged 13.3 -> 11.4); at N = 1536 (QKV, 3.1 vs 2.5 tiles
  // per CU) the 128-row ring stays faster (24.5 vs 27.6 us; scripts/dev/gemm_variants.py 9,10)
  const long long tn = (g.N + BN - 1) / BN;
  const long long t128 = (g.M + 127) / 128 * tn, t160 = (g.M + BM160 - 1) / BM160 * tn;
  const long long cu = tm_cu_count();
  return t128 > cu && t160 <= cu;
}

#ifdef TM_DIAG
// the persistent register-epilogue kernel (k-contiguous A, no split): diagnostic build only, variant
// 11 wherever valid (the product library never selects it: slower on every step shape)
inline bool use_pr(const tm_gemm_args& g) {
  if (g.a_trans || g.splits != 1 || g.K % 64 != 0 || g.mode == TM_EPI_SPLITK || g.pre_bf16) return false;
  if (g.b_kn && (g.N % 8 != 0 || g.N < 8)) return false;
  return GEMM_VARIANT == 11;
}
#endif

// the big-tile kernel's valid shapes; selected for every valid GEMM by diagnostic variant 7, and in the
// product for the to_qkv projection (head-major scatter epilogue, N >= 1024, no split): 198 tiles of
// 256 x 256 at n' = 8448 fill the chip in one round where the 128 x 128 ring needed 1.55 rounds of
// 792 tiles (microbench 23.2 vs 27.6 us; scripts/microbench.py --gemm-ab)
inline bool qkv_big_enabled() {   // TM_GEMM_QKV_BIG=0: the 128 x 128 ring for to_qkv (A/B runs only)
  static const bool on = [] { const char* e = std::getenv("TM_GEMM_QKV_BIG"); return !(e && e[0] == '0'); }();
  return on;
}
template <typename OutT>
bool big_ok(const tm_gemm_args& g) {
  const bool qkv_pick = (GEMM_VARIANT == 0 || GEMM_VARIANT == 12) && g.mode == TM_EPI_QKV && g.N >= 1024 && g.splits == 1 && g.M >= 2048 &&
                        !g.a_trans && !g.b_kn && qkv_big_enabled();
  if (GEMM_VARIANT != 7 && !qkv_pick) return false;
  if (g.K % 64 != 0 || (g.splits > 1 && g.k_per_split % 64 != 0)) return false;
  if (g.a_trans && (g.M % 8 != 0 || g.M < 8)) return false;
  if (g.b_kn && (g.N % 8 != 0 || g.N < 8)) return false;
  return g.M >= 128 && g.N >= 128;
}

template <typename T, typename OutT>
int launch_t(const void* A, const void* B, void* C, const tm_gemm_args& g, hipStream_t st) {
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, g.splits);
  if constexpr (sizeof(T) == 2) {
    if (big_ok<OutT>(g)) {
#ifdef TM_DIAG
#define TM_BIG_STAMP(AT, BKN, TBN)                                                                   \
      if (GEMM_VARIANT == 12) {   /* diagnostic: the QKV pick with per-workgroup stamps */         \
        tm_allow_smem(gemm_big_kernel<OutT, AT, BKN, TBN, true>, sm);                                \
        gemm_big_kernel<OutT, AT, BKN, TBN, true><<<gb, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
      } else
#else
#define TM_BIG_STAMP(AT, BKN, TBN)
#endif
#define TM_BIG_CASE(AT, BKN, TBN)                                                                  \
      if (g.a_trans == AT && g.b_kn == BKN) {                                                      \
        constexpr int sm = big_lds<OutT, TBN>();                                                   \
        tm_allow_smem(gemm_big_kernel<OutT, AT, BKN, TBN>, sm);                                   \
        const dim3 gb((g.N + TBN - 1) / TBN, (g.M + GBM - 1) / GBM, g.splits);                      \
        TM_BIG_STAMP(AT, BKN, TBN)                                                                 \
        gemm_big_kernel<OutT, AT, BKN, TBN><<<gb, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
        TM_CHECK_LAUNCH();                                                                         \
        return 0;                                                                                  \
      }
      if (g.N >= 1024) {
        TM_BIG_CASE(0, 0, 256) TM_BIG_CASE(0, 1, 256) TM_BIG_CASE(1, 0, 256) TM_BIG_CASE(1, 1, 256)
      } else {
        TM_BIG_CASE(0, 0, 128) TM_BIG_CASE(0, 1, 128) TM_BIG_CASE(1, 0, 128) TM_BIG_CASE(1, 1, 128)
      }
#undef TM_BIG_STAMP
#undef TM_BIG_CASE
    }
#ifdef TM_DIAG
    if (ring_ok<OutT>(g) && GEMM_VARIANT == 4) {
      const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
      const int ntiles = tiles_m * tiles_n * g.splits;
      const int nwg = ntiles < 256 ? ntiles : 256;
#define TM_PERSIST_CASE(AT, BKN)                                                                \
      if (g.a_trans == AT && g.b_kn == BKN) {                                                   \
        tm_allow_smem(gemm_persist_kernel<OutT, AT, BKN>, PERSIST_LDS);                         \
        gemm_persist_kernel<OutT, AT, BKN><<<nwg, 512, PERSIST_LDS, st>>>((const bf16*)A, (const bf16*)B, \
                                                                        (OutT*)C, g, tiles_m, tiles_n); \
        TM_CHECK_LAUNCH();                                                                      \
        return 0;                                                                               \
      }
      TM_PERSIST_CASE(0, 0) TM_PERSIST_CASE(0, 1) TM_PERSIST_CASE(1, 0) TM_PERSIST_CASE(1, 1)
#undef TM_PERSIST_CASE
    }
    if (use_pr(g)) {
      const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
      const int ntiles = tiles_m * tiles_n, cap = 2 * tm_cu_count();
      const int nwg = ntiles < cap ? ntiles : cap;
      const int kind = epilogue_kind(g);
#define TM_PR(BKN, K)                                                                                \
      {                                                                                              \
        tm_allow_smem(gemm_pr_kernel<OutT, BKN, K>, PR_LDS);                                         \
        gemm_pr_kernel<OutT, BKN, K><<<nwg, 512, PR_LDS, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g, \
                                                              tiles_m, tiles_n);                     \
      }
      if (g.b_kn) {
        if (kind == EK_PLAIN) TM_PR(true, EK_PLAIN) else if (kind == EK_QKV) TM_PR(true, EK_QKV) else TM_PR(true, EK_ANY)
      } else {
        if (kind == EK_PLAIN) TM_PR(false, EK_PLAIN) else if (kind == EK_QKV) TM_PR(false, EK_QKV) else TM_PR(false, EK_ANY)
      }
#undef TM_PR
      TM_CHECK_LAUNCH();
      return 0;
    }
#endif
    if (use_ring160(g)) {
      constexpr size_t sm = 2 * R160_STAGE;
      const dim3 g160((g.N + BN - 1) / BN, (g.M + BM160 - 1) / BM160);
      const int kind = epilogue_kind(g);
#define TM_R160(BKN, K)                                                                             \
      {                                                                                             \
        tm_allow_smem(gemm_ring160_kernel<OutT, BKN, K>, sm);                                       \
        gemm_ring160_kernel<OutT, BKN, K><<<g160, 640, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
      }
      if (g.b_kn) {
        if (kind == EK_PLAIN) TM_R160(true, EK_PLAIN) else if (kind == EK_QKV) TM_R160(true, EK_QKV) else TM_R160(true, EK_ANY)
      } else {
        if (kind == EK_PLAIN) TM_R160(false, EK_PLAIN) else if (kind == EK_QKV) TM_R160(false, EK_QKV) else TM_R160(false, EK_ANY)
      }
#undef TM_R160
      TM_CHECK_LAUNCH();
      return 0;
    }
    if (ring_ok<OutT>(g)) {
      constexpr size_t epi = (size_t)BM * EP_ROW * sizeof(float);
#ifdef TM_DIAG
#define TM_RING_DIAG(AT, BKN)                                                                   \
        else if (GEMM_VARIANT == 8) {                                                       \
          constexpr size_t sm = 2 * STAGE_BYTES > epi ? 2 * STAGE_BYTES : epi;                  \
          tm_allow_smem(gemm_ring_kernel<OutT, AT, BKN, 2, true>, sm);                          \
          gemm_ring_kernel<OutT, AT, BKN, 2, true><<<grid, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
        } else if (GEMM_VARIANT == 6) {                                                       \
          constexpr size_t sm = 3 * STAGE_BYTES > epi ? 3 * STAGE_BYTES : epi;                  \
          tm_allow_smem(gemm_ring_kernel<OutT, AT, BKN, 3>, sm);                                \
          gemm_ring_kernel<OutT, AT, BKN, 3><<<grid, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
        } else {                                                                                \
          constexpr size_t sm = RING_BYTES > epi ? RING_BYTES : epi;                            \
          tm_allow_smem(gemm_ring_kernel<OutT, AT, BKN>, sm);                                   \
          gemm_ring_kernel<OutT, AT, BKN><<<grid, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
        }
#else
#define TM_RING_DIAG(AT, BKN)
#endif
#define TM_RING_CASE(AT, BKN)                                                                   \
      if (g.a_trans == AT && g.b_kn == BKN) {                                                   \
        if (GEMM_VARIANT == 0 || GEMM_VARIANT == 5 || GEMM_VARIANT == 9) {                  \
          constexpr size_t sm = 2 * STAGE_BYTES > epi ? 2 * STAGE_BYTES : epi;                  \
          const int kind = epilogue_kind(g);                                                    \
          if (kind == EK_PLAIN) {                                                               \
            tm_allow_smem(gemm_ring_kernel<OutT, AT, BKN, 2, false, EK_PLAIN>, sm);             \
            gemm_ring_kernel<OutT, AT, BKN, 2, false, EK_PLAIN><<<grid, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
          } else if (kind == EK_QKV) {                                                          \
            tm_allow_smem(gemm_ring_kernel<OutT, AT, BKN, 2, false, EK_QKV>, sm);               \
            gemm_ring_kernel<OutT, AT, BKN, 2, false, EK_QKV><<<grid, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
          } else if (kind == EK_SPLITK) {                                                       \
            tm_allow_smem(gemm_ring_kernel<OutT, AT, BKN, 2, false, EK_SPLITK>, sm);            \
            gemm_ring_kernel<OutT, AT, BKN, 2, false, EK_SPLITK><<<grid, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
          } else {                                                                              \
            tm_allow_smem(gemm_ring_kernel<OutT, AT, BKN, 2>, sm);                              \
            gemm_ring_kernel<OutT, AT, BKN, 2><<<grid, 512, sm, st>>>((const bf16*)A, (const bf16*)B, (OutT*)C, g); \
          }                                                                                     \
        }                                                                                       \
        TM_RING_DIAG(AT, BKN)                                                                   \
        TM_CHECK_LAUNCH();                                                                      \
        return 0;                                                                               \
      }
      TM_RING_CASE(0, 0) TM_RING_CASE(0, 1) TM_RING_CASE(1, 0) TM_RING_CASE(1, 1)
#undef TM_RING_CASE
#undef TM_RING_DIAG
    }
  }
  const T* a = (const T*)A;
  const T* b = (const T*)B;
  OutT* c = (OutT*)C;
#ifdef TM_DIAG
#define TM_GEMM_2BUF(AT, BKN)                                                       \
    if (GEMM_VARIANT == 1) {                                                        \
      constexpr size_t sm = gemm_smem<T, AT, BKN>();                                \
      tm_allow_smem(gemm_kernel<T, OutT, AT, BKN>, sm);                             \
      gemm_kernel<T, OutT, AT, BKN><<<grid, 256, sm, st>>>(a, b, c, g);             \
      TM_CHECK_LAUNCH();                                                            \
      return 0;                                                                     \
    }
#else
#define TM_GEMM_2BUF(AT, BKN)
#endif
#define TM_GEMM_CASE(AT, BKN)                                                       \
  if (g.a_trans == AT && g.b_kn == BKN) {                                           \
    TM_GEMM_2BUF(AT, BKN)                                                           \
    constexpr size_t sm = gemm_smem<T, AT, BKN, 1>();                               \
    tm_allow_smem(gemm_kernel<T, OutT, AT, BKN, 1>, sm);                            \
    gemm_kernel<T, OutT, AT, BKN, 1><<<grid, 256, sm, st>>>(a, b, c, g);            \
    TM_CHECK_LAUNCH();                                                              \
    return 0;                                                                       \
  }
  TM_GEMM_CASE(0, 0) TM_GEMM_CASE(0, 1) TM_GEMM_CASE(1, 0) TM_GEMM_CASE(1, 1)
#undef TM_GEMM_CASE
#undef TM_GEMM_2BUF
  tm_set_error("gemm: bad transpose flags");
  return 1;
}

// out = alpha * sum_z slab[z] (+ out): the splits are summed in index order (bitwise
// reproducible).  U loads per thread are issued together (indices clamped, masked by
// select, no branches), so a 33-way reduce is one memory round trip, not five.
template <int U, int VEC>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                            int splits, size_t count, float alpha, int accumulate) {
  typedef float vf __attribute__((ext_vector_type(VEC)));
  const size_t iv = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (iv * VEC >= count) return;
  if (iv * VEC + VEC <= count) {
    vf s = (vf)0.f;
    for (int z0 = 0; z0 < splits; z0 += U) {
      vf v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *(const vf*)(slab + (size_t)min(z0 + u, splits - 1) * count + iv * VEC);
#pragma unroll
      for (int u = 0; u < U; ++u) s += (z0 + u < splits) ? v[u] : (vf)0.f;
    }
    s *= alpha;
    if (accumulate) s += *(const vf*)(out + iv * VEC);
    *(vf*)(out + iv * VEC) = s;
  } else {
    for (size_t i = iv * VEC; i < count; ++i) {
      float t = slab[i];
      for (int z = 1; z < splits; ++z) t += slab[(size_t)z * count + i];
      t *= alpha;
      if (accumulate) t += out[i];
      out[i] = t;
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
  if (c < cols) {
    // 8 independent partial sums per thread: eight row loads in flight at once
    float p8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int r = r0 + sub;
    for (; r + 28 < r1; r += 32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) p8[j] += to_f(X[(size_t)(r + 4 * j) * ld + c]);
    }
    for (; r < r1; r += 4) p8[0] += to_f(X[(size_t)r * ld + c]);
    s = ((p8[0] + p8[1]) + (p8[2] + p8[3])) + ((p8[4] + p8[5]) + (p8[6] + p8[7]));
  }
  red[sub][threadIdx.x & 63] = s;
  __syncthreads();
  if (sub == 0 && c < cols)
    part[(size_t)blockIdx.y * cols + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

}  // namespace

extern "C" int tm_gemm(const void* A, const void* B, void* C, const tm_gemm_args* g, void* stream) {
  TM_REQUIRE(g && A && B && C, "gemm: null argument");
  TM_REQUIRE(g->M >= 0 && g->N >= 0 && g->K >= 0 && g->splits >= 1, "gemm: bad shape");
  TM_REQUIRE(g->mode != TM_EPI_SPLITK || g->c_dtype == TM_F32, "gemm: split-K slabs are fp32 (or bf16 via slab_bf16)");
  TM_REQUIRE(!g->slab_bf16 || (g->mode == TM_EPI_SPLITK && g->ab_dtype == TM_BF16),
             "gemm: slab_bf16 is for bf16 split-K weight gradients");
  TM_REQUIRE(g->k_per_split > 0, "gemm: k_per_split must be > 0");
  TM_REQUIRE(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "gemm: operands must be 16-B aligned");
  const int E = g->ab_dtype == TM_BF16 ? 8 : 4;
  TM_REQUIRE(g->lda % E == 0 && g->ldb % E == 0, "gemm: leading dimensions must be multiples of 16 B");
  TM_REQUIRE(g->mode != TM_EPI_QKV || (g->dh % 8 == 0 && g->N % 8 == 0), "gemm: QKV scatter needs dh % 8 == 0");
  if (g->M == 0 || g->N == 0) return 0;
  // the fused bias-gradient column sums ride in the bf16 ring kernel's split-K weight-gradient form only
  TM_REQUIRE(!g->colsum || (g->ab_dtype == TM_BF16 && g->c_dtype == TM_F32 && g->a_trans && g->mode == TM_EPI_SPLITK &&
                            ring_ok<float>(*g) && (GEMM_VARIANT == 0 || GEMM_VARIANT == 5 || GEMM_VARIANT == 9)),
             "gemm: colsum needs the bf16 split-K weight-gradient ring path (a_trans, K % 64 == 0, M % 8 == 0)");
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

#ifdef TM_DIAG
extern "C" void tm_debug_set_gemm_variant(int value) { g_gemm_variant = value; }

// copy the variant-8 ring stamps ([block][8] u64) to a host buffer (diagnostics only)
extern "C" int tm_debug_gemm_stamps(unsigned long long* host, int count) {
  TM_REQUIRE(count > 0 && count <= 2048 * 8, "gemm_stamps: bad count");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_stamps), count * sizeof(unsigned long long)) != hipSuccess) {
    tm_set_error("gemm_stamps: copy");
    return 1;
  }
  return 0;
}
#endif

// ---- deferred reductions: the parameter-gradient slab sums of a backward, queued in a
// CALLER-OWNED tm_reduce_queue and summed by ONE launch at tm_reduce_flush (a kernel boundary
// costs ~4.5 us in graph replay on gfx950; a backward has ~15 such sums that nothing reads before
// the optimizer).  Same fixed split order as splitk_reduce_kernel, so results are bit-identical.
// The library keeps no deferral state of its own: every engine / thread / stream passes its own
// queue (or NULL = launch now), so concurrent callers never see each other's entries.
namespace {
constexpr int DEFER_MAX = 48;
struct ReduceEntry {
  const void* slab;  // fp32, or bf16 (bf16 != 0: the bf16-mode attention partial slabs)
  float* out;
  long long count;
  int splits;
  int accumulate;
  float alpha;
  int vec;   // 1: 4-element units (count % 4 == 0, aligned); 2: bf16 slabs in 8-element units (16-B loads)
  int par;   // threads per output unit (power of 2 <= 64): each sums every par-th split, then a
             // fixed xor-shuffle tree (entries with many splits and few outputs, e.g. LayerNorm
             // weight partials of every 32-row block, would otherwise be one long serial loop)
  int bf16;  // slab elements are bf16 (summed in fp32 like the fp32 ones, same order)
};
struct ReduceTable {
  ReduceEntry e[DEFER_MAX];
  long long off[DEFER_MAX + 1];   // prefix sums of the entries' thread counts
  int boff[DEFER_MAX + 1];        // prefix sums of the entries' workgroup counts (256 threads each)
  int n;
};
static_assert(sizeof(ReduceTable) <= 4096, "multi_reduce_kernel's table must fit the kernel-argument segment");

}  // namespace

struct tm_reduce_queue {
  unsigned magic;
  ReduceTable t;
};

namespace {
constexpr unsigned RQ_MAGIC = 0x52514D54u;   // "TMQR"

// one thread = one 16-B unit (4 floats; entries whose count is not a multiple of 4 or whose
// pointers are not 16-B aligned go element by element); every workgroup lies inside one entry
// (found once per workgroup through the scalar path), the splits summed in index order with
// 12 loads in flight per thread
__global__ __launch_bounds__(256) void multi_reduce_kernel(ReduceTable t) {
  int e = 0;
  while ((int)blockIdx.x >= t.boff[e + 1]) ++e;
  const ReduceEntry r = t.e[e];
  const long long tt = (long long)(blockIdx.x - t.boff[e]) * 256 + threadIdx.x;
  if (tt >= t.off[e + 1] - t.off[e]) return;  // whole groups of par lanes (par | 64) leave together
  const int par = r.par, sub = (int)(tt & (par - 1));
  const long long u = tt / par;
  constexpr int U = 12;
  if (r.vec == 2) {   // bf16 slabs, 8 elements (one 16-B load) per unit: as many bytes in flight as fp32
    const size_t j = (size_t)u * 8;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
    for (int z0 = sub; z0 < r.splits; z0 += U * par) {
      bf16x8 v[U];
#pragma unroll
      for (int k = 0; k < U; ++k)
        v[k] = *(const bf16x8*)((const bf16*)r.slab + (size_t)min(z0 + k * par, r.splits - 1) * r.count + j);
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (z0 + k * par < r.splits) {
          s0 += (f32x4){(float)v[k][0], (float)v[k][1], (float)v[k][2], (float)v[k][3]};
          s1 += (f32x4){(float)v[k][4], (float)v[k][5], (float)v[k][6], (float)v[k][7]};
        }
    }
    for (int o = 1; o < par; o <<= 1)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        s0[c] += __shfl_xor(s0[c], o, 64);
        s1[c] += __shfl_xor(s1[c], o, 64);
      }
    if (sub) return;
    s0 *= r.alpha;
    s1 *= r.alpha;
    if (r.accumulate) {
      s0 += *(const f32x4*)(r.out + j);
      s1 += *(const f32x4*)(r.out + j + 4);
    }
    *(f32x4*)(r.out + j) = s0;
    *(f32x4*)(r.out + j + 4) = s1;
    return;
  }
  if (r.vec) {
    const size_t j = (size_t)u * 4;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int z0 = sub; z0 < r.splits; z0 += U * par) {
      f32x4 v[U];
      if (r.bf16) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const bf16x4 b = *(const bf16x4*)((const bf16*)r.slab + (size_t)min(z0 + k * par, r.splits - 1) * r.count + j);
          v[k] = (f32x4){(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
        }
      } else {
#pragma unroll
        for (int k = 0; k < U; ++k)
          v[k] = *(const f32x4*)((const float*)r.slab + (size_t)min(z0 + k * par, r.splits - 1) * r.count + j);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) s += (z0 + k * par < r.splits) ? v[k] : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    for (int o = 1; o < par; o <<= 1)
#pragma unroll
      for (int c = 0; c < 4; ++c) s[c] += __shfl_xor(s[c], o, 64);
    if (sub) return;
    s *= r.alpha;
    if (r.accumulate) s += *(const f32x4*)(r.out + j);
    *(f32x4*)(r.out + j) = s;
    return;
  }
  float s = 0.f;
  for (int z0 = sub; z0 < r.splits; z0 += U * par) {
    float v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const size_t idx = (size_t)min(z0 + k * par, r.splits - 1) * r.count + u;
      v[k] = r.bf16 ? (float)((const bf16*)r.slab)[idx] : ((const float*)r.slab)[idx];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) s += (z0 + k * par < r.splits) ? v[k] : 0.f;
  }
  for (int o = 1; o < par; o <<= 1) s += __shfl_xor(s, o, 64);
  if (sub) return;
  s *= r.alpha;
  if (r.accumulate) s += r.out[u];
  r.out[u] = s;
}
}  // namespace

extern "C" tm_reduce_queue* tm_reduce_queue_create(void) {
  tm_reduce_queue* q = new (std::nothrow) tm_reduce_queue{};
  if (!q) {
    tm_set_error("reduce_queue_create: out of host memory");
    return nullptr;
  }
  q->magic = RQ_MAGIC;
  return q;
}

extern "C" void tm_reduce_queue_destroy(tm_reduce_queue* q) {
  if (q && q->magic == RQ_MAGIC) {
    q->magic = 0;
    delete q;
  }
}

extern "C" int tm_reduce_queue_pending(const tm_reduce_queue* q) {
  return (q && q->magic == RQ_MAGIC) ? q->t.n : -1;
}

extern "C" int tm_reduce_flush(tm_reduce_queue* q, void* stream) {
  TM_REQUIRE(q && q->magic == RQ_MAGIC, "reduce_flush: not a tm_reduce_queue");
  ReduceTable& t = q->t;
  if (t.n == 0) return 0;
  t.boff[0] = 0;
  for (int i = 0; i < t.n; ++i)
    t.boff[i + 1] = t.boff[i] + (int)((t.off[i + 1] - t.off[i] + 255) / 256);
  multi_reduce_kernel<<<(unsigned)t.boff[t.n], 256, 0, (hipStream_t)stream>>>(t);
  t.n = 0;
  t.off[0] = 0;
  TM_CHECK_LAUNCH();
  return 0;
}

namespace {
// one multi_reduce entry appended to t (the caller has made room)
void push_reduce_entry(ReduceTable& t, const void* slab, int slab_bf16, float* out, int splits, long long count,
                       float alpha, int accumulate) {
  // vec 2: bf16 slabs in 8-element units (16-B loads); 1: 4-element units; 0: element by element
  const int vec = slab_bf16 && count % 8 == 0 && ((uintptr_t)slab % 16) == 0 && ((uintptr_t)out % 16) == 0
                      ? 2
                      : (count % 4 == 0 && ((uintptr_t)slab % (slab_bf16 ? 8 : 16)) == 0 && ((uintptr_t)out % 16) == 0);
  const long long units = vec == 2 ? count / 8 : vec ? count / 4 : count;
  // threads per unit: enough that each sums <= 2 bursts of 12 splits, while the entry keeps
  // to <= ~64 K threads
  int par = 1;
  while (par < 64 && (splits + par - 1) / par > 24 && units * par * 2 <= 65536) par <<= 1;
  t.e[t.n] = ReduceEntry{slab, out, count, splits, accumulate, alpha, vec, par, slab_bf16};
  // offsets count threads: par per 16-B unit (or element)
  t.off[t.n + 1] = t.off[t.n] + units * par;
  ++t.n;
}
}  // namespace

// Library-internal (not in the ABI header): the split-K sum of a slab of fp32 or bf16 partials
// (slab_dtype TM_F32 / TM_BF16), deferred into q when given.  The bf16 form serves the bf16-mode
// attention backward's partial slabs; both forms add the splits in index order in fp32.
int tm_splitk_reduce_typed(const void* slab, int slab_dtype, float* out, int splits, long long count, float alpha,
                           int accumulate, tm_reduce_queue* q, void* stream) {
  if (slab_dtype == TM_F32)
    return tm_splitk_reduce((const float*)slab, out, splits, count, alpha, accumulate, q, stream);
  TM_REQUIRE(slab && out && splits >= 1 && count >= 0, "splitk_reduce: bad args");
  TM_REQUIRE(!q || q->magic == RQ_MAGIC, "splitk_reduce: not a tm_reduce_queue");
  if (count == 0) return 0;
  if (q) {
    if (q->t.n == DEFER_MAX)
      if (int rc = tm_reduce_flush(q, stream)) return rc;
    push_reduce_entry(q->t, slab, 1, out, splits, count, alpha, accumulate);
    return 0;
  }
  tm_reduce_queue local{};   // not deferred: a one-entry table launched now
  local.magic = RQ_MAGIC;
  push_reduce_entry(local.t, slab, 1, out, splits, count, alpha, accumulate);
  return tm_reduce_flush(&local, stream);
}

extern "C" int tm_splitk_reduce_bf16(const void* slab, float* out, int splits, long long count, float alpha,
                                     int accumulate, tm_reduce_queue* q, void* stream) {
  return tm_splitk_reduce_typed(slab, TM_BF16, out, splits, count, alpha, accumulate, q, stream);
}

extern "C" int tm_splitk_reduce(const float* slab, float* out, int splits, long long count, float alpha,
                                int accumulate, tm_reduce_queue* q, void* stream) {
  TM_REQUIRE(slab && out && splits >= 1 && count >= 0, "splitk_reduce: bad args");
  TM_REQUIRE(!q || q->magic == RQ_MAGIC, "splitk_reduce: not a tm_reduce_queue");
  if (count == 0) return 0;
  if (q) {
    if (q->t.n == DEFER_MAX)
      if (int rc = tm_reduce_flush(q, stream)) return rc;
    push_reduce_entry(q->t, slab, 0, out, splits, count, alpha, accumulate);
    return 0;
  }
  hipStream_t st = (hipStream_t)stream;
  // float4 per thread only when that still gives >= 1024 workgroups' worth of threads
  const bool vec4 = count % 4 == 0 && count / 4 >= 256LL * 1024;
  const size_t nthreads = vec4 ? (size_t)count / 4 : (size_t)count;
  const unsigned blocks = (unsigned)((nthreads + 255) / 256);
  if (splits <= 8) {
    if (vec4) splitk_reduce_kernel<8, 4><<<blocks, 256, 0, st>>>(slab, out, splits, (size_t)count, alpha, accumulate);
    else splitk_reduce_kernel<8, 1><<<blocks, 256, 0, st>>>(slab, out, splits, (size_t)count, alpha, accumulate);
  } else if (splits <= 16) {
    if (vec4) splitk_reduce_kernel<16, 4><<<blocks, 256, 0, st>>>(slab, out, splits, (size_t)count, alpha, accumulate);
    else splitk_reduce_kernel<16, 1><<<blocks, 256, 0, st>>>(slab, out, splits, (size_t)count, alpha, accumulate);
  } else {
    if (vec4) splitk_reduce_kernel<36, 4><<<blocks, 256, 0, st>>>(slab, out, splits, (size_t)count, alpha, accumulate);
    else splitk_reduce_kernel<36, 1><<<blocks, 256, 0, st>>>(slab, out, splits, (size_t)count, alpha, accumulate);
  }
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_colsum_workspace(int rows, int cols, int rows_per_chunk) {
  const int nchunk = (rows + rows_per_chunk - 1) / rows_per_chunk;
  return (long long)nchunk * cols * (long long)sizeof(float);
}

// out[c] (+)= sum_r X[r, c]; deterministic two-level sum through `work`
extern "C" int tm_colsum(const void* X, int dtype, int rows, int cols, int ld, int rows_per_chunk, float* work,
                         float* out, int accumulate, tm_reduce_queue* rq, void* stream) {
  TM_REQUIRE(X && work && out && rows_per_chunk > 0, "colsum: bad args");
  const int nchunk = (rows + rows_per_chunk - 1) / rows_per_chunk;
  dim3 grid((cols + 63) / 64, nchunk);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16)
    colsum_partial_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)X, rows, cols, ld, rows_per_chunk, work);
  else
    colsum_partial_kernel<float><<<grid, 256, 0, st>>>((const float*)X, rows, cols, ld, rows_per_chunk, work);
  TM_CHECK_LAUNCH();
  return tm_splitk_reduce(work, out, nchunk, cols, 1.0f, accumulate, rq, stream);
}
