// Moore-Penrose iterative pseudo-inverse (SURVEY.md App. A eq. 7) for the bf16 (bench) mode:
// the chain of moore_penrose_iter_pinv (third-party nystrom_attention, called from
// NystromAttention.forward, code/models/TransMIL.py:47) and its backward, on "split" operands.
//
// Split storage.  Every 256x256 chain matrix M of B*h heads is kept as two bf16 planes,
// hi = bf16(M) and lo = bf16(M - hi) (lo plane at hi + nbh*65536 elements; the pair takes the
// bytes of one fp32 matrix and holds M to ~2^-17 relative).  A product C = op(A) op(B) is
// hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16 with fp32 accumulation ("bf16x3"), so the
// operands feed the MFMA straight from LDS: no per-fragment fp32 -> bf16 split in the consumer.
//
// Stage kernel.  One launch = up to three independent jobs (products of 1-2 terms, or the
// abs-sum reduction), each over all heads.  Workgroup = one 64x64 output tile of one head,
// 8 waves: 2x2 subtiles of 32x32, each subtile's k-steps split over the two waves of one SIMD
// (partial tiles summed in the epilogue), the whole K of every term.  Operand chunks (64 rows x 64 k, hi and lo)
// come by LDS-DMA (global_load_lds, 16 B per lane, no VGPR round trip) into a 3-slot ring of
// 32 KB, two chunks ahead of the MFMAs (counted s_waitcnt vmcnt + raw s_barrier).  LDS images:
//   "kc" (k-contiguous: the stored row is the output index, op(A) = A or op(B) = B^T):
//       [64 rows][64 k], 16-B slot c of row r at c ^ ((r >> 1) & 7)  -> ds_read_b128 fragments
//   "kr" (k-rows: the stored row is k, op(A) = A^T or op(B) = B):
//       [64 k][64 cols], slot c of k-row k at c ^ (((k >> 1) & 1) << 2) -> 2 x ds_read_b64_tr_b16
// (both bank-conflict free; the swizzle is applied to the DMA source address).  The epilogue
// stages the fp32 tile through LDS and writes whole 16-B row pieces: scale, diagonal, up to two
// addend matrices, and up to four outputs (split, fp32, and two split side outputs).
//
// Forward schedule (P_k = X Z_k, carried by its own recurrence, as in pinv.hip), per layer:
//   L1:  S = X X^T                       + |X| row / column sums, per-head maxima
//   A_0: R = S S / c^2,  T3 = R - 7 S/c + 15I,  P_0 = S/c          (c = max rowsum * max colsum)
//   B_k: T5 = 13I - P T3,  P_{k+1} = 3.25 P - 0.25 R T3
//   A_k: R = P P, T3 = R - 7P + 15I,  Z_k = 0.25 Z_{k-1} T5_{k-1}  (Z_0 = X^T / c is never formed)
//   F:   Z_6 = 0.25 Z_5 T5_5  (split + fp32)
// 14 dependent launches.  The backward runs the reference graph's adjoint (4 launches per
// iteration), then one launch for the partial sums of the c gradient and one that applies the
// Z_0 = X^T / c terms and (optionally) the softmax backward of A2 = X.
#include "common.h"
#include "a3_combine.h"
#include "../../include/transmil_hip.h"

namespace {

constexpr int NL = 256;
constexpr int MAT = NL * NL;            // elements per head matrix
constexpr int PC = 64 * 128;            // one 64 x 64 bf16 plane chunk image: 8 KB
constexpr int SLOT = 4 * PC;            // A hi, A lo, B hi, B lo
constexpr int NSLOT = 3;
constexpr int STAGE_LDS = NSLOT * SLOT; // 96 KB ring
constexpr int EROW = 68;                // epilogue tile row (floats)
constexpr int EPI_LDS = 64 * EROW * 4;  // the fp32 output tile (17 KB); one workgroup per CU
constexpr int MAXJ = 3;
constexpr int NPROD = 8;                // producer (LDS-DMA) waves; 4 consumer waves
constexpr int NTHREADS = 64 * (4 + NPROD);
// persistent chain kernel (pinv_team_kernel): per XCD a ticket and a done counter on their own
// 64-B lines, then one error word; a forward and a backward set live at the end of `saved`
constexpr int TEAM_XCD = 8;
constexpr int TEAM_STRIDE = 16;                          // u32 words between two XCDs' counters
constexpr int TEAM_SET_WORDS = TEAM_XCD * TEAM_STRIDE + 16;
constexpr int TEAM_CTR_WORDS = 2 * TEAM_SET_WORDS;

typedef __attribute__((address_space(3))) void lds_t;
typedef __attribute__((address_space(1))) void glb_t;
typedef __attribute__((address_space(3))) bf16x4 lds_v4;

struct SOp {
  const bf16* p;  // hi plane of head 0 (lo plane at p + plane)
  int kr;         // 1: stored row index is k ("kr" image), 0: stored row is the output index ("kc")
  int pad;
};

enum { KIND_PRODUCT = 0, KIND_ABSSUMS = 1 };

struct SJob {
  SOp a[2], b[2];
  int nterms, kind;
  float alpha, diag;       // s = alpha * invc^alpha_cpow * sum;  v = s + diag*I + e1s*E1' + e2s*E2
  int alpha_cpow, e1_cpow; // E1' = E1 * invc^e1_cpow
  const void* e1; float e1s; int e1_f32;
  const void* e2; float e2s; int e2_f32;
  void* c; int c_f32; int pad0;
  float* cf;                                // optional fp32 copy of v
  bf16* c2; float c2_alpha, c2_diag, c2_e1; // optional split: c2_alpha*s + c2_diag*I + c2_e1*E1'
  bf16* c3; float c3_e1; int pad1;          // optional split: c3_e1 * E1'
};
// The DOT stage-kernel instantiation (the backward's last level only) reads its job's e2 as
// `dotx` (fp32, head-major like the output; that job has no E2 addend) and cf as `dot_part`: the
// workgroup's partial of sum_ij v[i][j] dotx[j][i] at dot_part[head * 16 + tile] -- the c
// gradient's dot without a separate launch, and without growing every launch's kernel arguments.
TM_DEV const float* job_dotx(const SJob& J) { return (const float*)J.e2; }
TM_DEV float* job_dot_part(const SJob& J) { return J.cf; }

struct SLaunch {
  SJob j[MAXJ];
  int njobs, nbh;
  long long plane;          // elements between the hi and lo planes of a split matrix
  const float* maxima;      // [2][nbh] per-head maxima of the |X| row / column sums (for invc), or null
  const float* X;           // fp32 X (abs-sum jobs)
  float* sums;              // [2][nbh][256] row / column sums (abs-sum jobs)
  float* maxima_out;        // [2][nbh] (abs-sum jobs)
  unsigned* zero_ctr;       // abs-sum launch: the team kernels' counters to zero (TEAM_CTR_WORDS), or null
  A3Combine a3;             // a3.w non-null: the row blockIdx.y == njobs runs the A3 forward's partial
                            // combine (a3_combine.h) on the CUs the chain's tiles leave idle
  int dbg;                  // ablation (microbench only): 1 no DMA, 2 no LDS reads / MFMA, 3 no epilogue,
                            // 4 epilogue only, 5 empty
  unsigned long long* stamps;  // diagnostic build only: per-wave s_memtime stamps, or null
};

#ifdef TM_DIAG
int g_split_dbg = 0;
unsigned long long* g_split_stamps = nullptr;
#define SPLIT_DBG (dbg_)
#define SPLIT_STAMPS (stamp_out != nullptr)
#else
#define SPLIT_DBG 0
#define SPLIT_STAMPS false
#endif

// one s_memtime stamp (shader clock), its own lgkmcnt wait inside the statement
TM_DEV unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
TM_DEV unsigned long long rstamp() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

TM_DEV float powc(float c, int p) { return p == 0 ? 1.f : (p == 1 ? c : c * c); }

// 1 / (max_all rowsum * max_all colsum) from the per-head maxima
// (scalar loads through the constant address space: no VMEM counter traffic, so the DMA ring's
// counted waits are not disturbed)
TM_DEV float inv_c(const float* maxima, int nbh) {
  typedef const __attribute__((address_space(4))) float cfloat;
  cfloat* m = (cfloat*)(uintptr_t)maxima;
  float mc = -INFINITY, mr = -INFINITY;
  for (int h = 0; h < nbh; ++h) { mc = fmaxf(mc, m[h]); mr = fmaxf(mr, m[nbh + h]); }
  return 1.f / (mc * mr);
}

// LDS reads as inline asm: hipcc (ROCm 7.2) puts an `s_waitcnt vmcnt(0)` in front of every
// ds_read_b64_tr_b16 builtin while an LDS-DMA is in flight (it cannot tell the DMA's target from
// the read's), which would drain the prefetch ring every k-step.  The asm reads are ordered by
// explicit lgkmcnt waits + sched_barrier (hipcc does not count them).
TM_DEV unsigned lds_off(const void* p) { return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p; }
template <int OFF> TM_DEV void ds_b128(bf16x8& d, unsigned a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}
template <int OFF> TM_DEV void ds_tr(bf16x4& d, unsigned a) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}
template <int N> TM_DEV void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// "kc" image: lane address of k-step s (rows ob + (lane&31), 16-B chunk 2s + (lane>>5))
TM_DEV unsigned kc_addr(int ob, int s, int lane) {
  const int r = ob + (lane & 31), c = 2 * s + (lane >> 5);
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}
// "kr" image: lane address of k-step 0, first 4 k-rows (16-lane group g: lane 4q+p -> k-row 8(g>>1)+q,
// outputs ob + 16(g&1) + 4p..+3); k-step s adds 16 rows (2048 B), the second 4 rows 512 B.
TM_DEV unsigned kr_addr(int ob, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int o = ob + (g & 1) * 16 + 4 * p;
  const int k = 8 * (g >> 1) + q;
  const int c = o >> 3, half = (o >> 2) & 1;
  return k * 128 + ((c ^ (((k >> 1) & 1) << 2)) << 4) + half * 8;
}

struct Frag { bf16x8 h, l; };
TM_DEV bf16x8 join(const bf16x4& a, const bf16x4& b) { return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }

// issue the LDS reads of one operand's (hi, lo) fragments of k-step S; PL = plane pair (0 A, 2 B)
template <int KR, int S, int PL>
TM_DEV void read_op(Frag& f, unsigned krbase, const unsigned (&kc)[4]) {
  if constexpr (KR) {
    bf16x4 a, b, c, d;
    ds_tr<PL * PC + S * 2048>(a, krbase);
    ds_tr<PL * PC + S * 2048 + 512>(b, krbase);
    ds_tr<(PL + 1) * PC + S * 2048>(c, krbase);
    ds_tr<(PL + 1) * PC + S * 2048 + 512>(d, krbase);
    f.h = join(a, b);
    f.l = join(c, d);
  } else {
    ds_b128<PL * PC>(f.h, kc[S]);
    ds_b128<(PL + 1) * PC>(f.l, kc[S]);
  }
}

// One 64-deep chunk of one term from ring slot `sb` (byte offset), by one consumer wave (its
// 32x32 subtile): 4 k-steps of 3 MFMAs, the LDS reads of step s+1 in flight during step s.
template <int AKR, int BKR>
TM_DEV void chunk_mma(f32x16& acc, unsigned sb, unsigned akr, unsigned bkr, const unsigned (&akc0)[4],
                      const unsigned (&bkc0)[4]) {
  constexpr int RS = (AKR ? 4 : 2) + (BKR ? 4 : 2);  // LDS reads per k-step
  unsigned akc[4], bkc[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) { akc[s] = akc0[s] + sb; bkc[s] = bkc0[s] + sb; }
  const unsigned ab = akr + sb, bb = bkr + sb;
  Frag a[2], b[2];
  read_op<AKR, 0, 0>(a[0], ab, akc); read_op<BKR, 0, 2>(b[0], bb, bkc);
  read_op<AKR, 1, 0>(a[1], ab, akc); read_op<BKR, 1, 2>(b[1], bb, bkc);
  wait_lgkm<RS>();
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0].l, b[0].h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0].h, b[0].l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0].h, b[0].h, acc, 0, 0, 0);
  read_op<AKR, 2, 0>(a[0], ab, akc); read_op<BKR, 2, 2>(b[0], bb, bkc);
  wait_lgkm<RS>();
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1].l, b[1].h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1].h, b[1].l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1].h, b[1].h, acc, 0, 0, 0);
  read_op<AKR, 3, 0>(a[1], ab, akc); read_op<BKR, 3, 2>(b[1], bb, bkc);
  wait_lgkm<RS>();
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0].l, b[0].h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0].h, b[0].l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0].h, b[0].h, acc, 0, 0, 0);
  wait_lgkm<0>();
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1].l, b[1].h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1].h, b[1].l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1].h, b[1].h, acc, 0, 0, 0);
}

template <int N>
TM_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// 8 consecutive elements of a split matrix as fp32
TM_DEV void load_split8(const bf16* hi, long long plane, size_t off, float* v) {
  const bf16x8 h = *(const bf16x8*)(hi + off), l = *(const bf16x8*)(hi + plane + off);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)h[e] + (float)l[e];
}
// 16-B store; wt: write-through (buffer_store sc1: the line goes out now and leaves this XCD's L2,
// so the launch-end L2 write-back has nothing of it to write)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
TM_DEV void st16(void* base, size_t off_bytes, f32x4 v, bool wt) {
  if (wt)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), tm_rsrc(base, 0x7FFFFFF0u),
                                           (unsigned)off_bytes, 0, 16);
  else
    *(f32x4*)((char*)base + off_bytes) = v;
}
TM_DEV void store_split8(bf16* hi, long long plane, size_t off, const float* v, bool wt = false) {
  bf16x8 h, l;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = (bf16)v[e];
    l[e] = (bf16)(v[e] - (float)h[e]);
  }
  st16(hi, off * 2, __builtin_bit_cast(f32x4, h), wt);
  st16(hi, (plane + off) * 2, __builtin_bit_cast(f32x4, l), wt);
}
TM_DEV void load_f8(const float* p, size_t off, float* v) {
  const f32x4 a = *(const f32x4*)(p + off), b = *(const f32x4*)(p + off + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
TM_DEV void store_f8(float* p, size_t off, const float* v, bool wt = false) {
  st16(p, off * 4, (f32x4){v[0], v[1], v[2], v[3]}, wt);
  st16(p, (off + 4) * 4, (f32x4){v[4], v[5], v[6], v[7]}, wt);
}

// |X| row sums (which = 0) or column sums (which = 1) of one head, and their maximum
// (threads 0..255 work, the other waves only meet the barriers)
TM_DEV void abssums(const SLaunch& L, int head, int which, float* red) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const bool on = t < NL;
  const float* x = L.X + (size_t)head * MAT;
  float s = 0.f;
  if (which == 0) {
    // wave w < 4: rows 64w..64w+63; lane l sums columns 4l..4l+3 of each row, the row total via LDS
    float* part = red + 16 + (wave & 3) * 64 * 65;
    if (on)
      for (int r = 0; r < 64; ++r) {
        const f32x4 v = *(const f32x4*)(x + (size_t)(wave * 64 + r) * NL + lane * 4);
        part[r * 65 + lane] = fabsf(v[0]) + fabsf(v[1]) + fabsf(v[2]) + fabsf(v[3]);
      }
    __syncthreads();
    if (on)
      for (int l = 0; l < 64; ++l) s += part[lane * 65 + l];
    // thread t now holds the sum of row 64*wave + lane = t
  } else if (on) {
    for (int i = 0; i < NL; ++i) s += fabsf(x[(size_t)i * NL + t]);
  }
  if (on) L.sums[((size_t)which * L.nbh + head) * NL + t] = s;
  const float m = wave_max(s);
  if (lane == 0 && on) red[wave] = m;
  __syncthreads();
  if (t == 0) L.maxima_out[which * L.nbh + head] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// Roles: waves 0-3 are consumers (one 32x32 subtile each, the whole K: LDS reads + MFMAs +
// epilogue), waves 4-7 producers (wave 4+p issues plane p of every chunk by LDS-DMA: 0 A hi,
// 1 A lo, 2 B hi, 3 B lo).  One s_barrier per chunk: a chunk is read after the barrier that
// follows its producers' counted vmcnt wait, and its slot is refilled after the barrier that
// follows the consumers' last read of it.
// TEAM: the tile runs inside the persistent chain kernel (pinv_team_kernel): every operand it
// reads was written by another workgroup of the same XCD in this launch, so the LDS-DMA reads
// bypass the CU's L1 (sc1, served by the XCD's L2) and so do the epilogue operand loads (nt).
template <bool TEAM, int TEAM_POL = 16, bool DOT = false>
TM_DEV void stage_tile(const SJob& J, int nbh, long long plane, const float* maxima, int head, int tile,
                       char* smem, unsigned long long* stamp_out, int dbg_, bool dj = false) {
  constexpr int DMA_POL = TEAM ? TEAM_POL : 0;   // cache policy of the LDS-DMA: sc1 in the team kernel
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = (tile >> 2) * 64, n0 = (tile & 3) * 64;
  const size_t hoff = (size_t)head * MAT;
  const int nch = J.nterms * 4;
  const int nchl = SPLIT_DBG == 4 ? 0 : nch;
  const bool st_on = SPLIT_STAMPS;
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (st_on) { ts[0] = rstamp(); ts[1] = stamp(); }

  // epilogue operands first (plain loads, issued before any DMA: every later counted wait covers
  // them): this thread's 8-element row piece (row tid/8, cols 8 (tid&7)) of E1 / E2, raw 16-B words
  const int lr = tid >> 3, lc = (tid & 7) * 8;
  const size_t eoff = hoff + (size_t)(m0 + lr) * NL + n0 + lc;
  const void* e1p = J.e1;
  const void* e2p = J.e2;
  const int e1f = J.e1_f32, e2f = J.e2_f32;
  f32x4 e1raw[2], e2raw[2];
  auto ld4 = [&](const f32x4* a) {
    if constexpr (TEAM) return __builtin_nontemporal_load(a);   // L1 bypass (written in this launch)
    else return *a;
  };
  auto eload = [&](const void* e, int f32, f32x4 (&r)[2]) {
    if (f32) {
      const float* q = (const float*)e;
      r[0] = ld4((const f32x4*)(q + eoff)); r[1] = ld4((const f32x4*)(q + eoff + 4));
    } else {
      const bf16* q = (const bf16*)e;
      r[0] = ld4((const f32x4*)(q + eoff)); r[1] = ld4((const f32x4*)(q + plane + eoff));
    }
  };
  const bool epi = tid < 512;  // the 512 threads that each own one 8-element piece of the 64x64 tile
  if (e1p && epi) eload(e1p, e1f, e1raw);
  const bool dotj = DOT && dj;   // this job carries the c-gradient dot in e2 / cf (job_dotx)
  if (!dotj && e2p && epi) eload(e2p, e2f, e2raw);
  // the transposed dotx piece of this thread's 8 outputs: dotx[col + e][row] (DOT: a separate
  // instantiation for the one launch that carries it, so the other levels keep their registers)
  float dxv[8];
  if (dotj && epi) {
    const float* dotx = job_dotx(J);
#pragma unroll
    for (int e = 0; e < 8; ++e) dxv[e] = dotx[hoff + (size_t)(n0 + lc + e) * NL + m0 + lr];
  }
  // per-head maxima for 1/c: one raw vector load per lane now, reduced in the epilogue
  const bool need_c = J.alpha_cpow || J.e1_cpow;
  float mcv = -INFINITY, mrv = -INFINITY;
  if (need_c && nbh <= 64 && lane < nbh) { mcv = maxima[lane]; mrv = maxima[nbh + lane]; }
  float* ep = (float*)(smem + STAGE_LDS);  // [64][EROW] fp32 tile for the epilogue

  if (wv >= 4) {  // ------------------------------------------------------------ producer
    // producer p = wv - 4 (0..NPROD-1) stages image rows of plane p / (NPROD/4) (0 A hi, 1 A lo,
    // 2 B hi, 3 B lo): PPW pieces of 8 rows each, starting at row 8 * PPW * (p % (NPROD/4))
    constexpr int PPW = 32 / NPROD;
    const int p = wv - 4, pl = p / (NPROD / 4), rb = (p % (NPROD / 4)) * PPW * 8;
    const SOp op0 = pl < 2 ? J.a[0] : J.b[0];
    const SOp op1 = pl < 2 ? J.a[1] : J.b[1];
    const int o0w = pl < 2 ? m0 : n0;
    const bf16* const pb0 = op0.p + hoff + ((pl & 1) ? plane : 0);
    const bf16* const pb1 = op1.p + hoff + ((pl & 1) ? plane : 0);
    unsigned loff[2][PPW];  // [kr][piece]: row * 256 + 8 * (slot ^ swizzle(row))
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int row = rb + i * 8 + (lane >> 3), pos = lane & 7;
      loff[0][i] = row * NL + 8 * (pos ^ ((row >> 1) & 7));
      loff[1][i] = row * NL + 8 * (pos ^ (((row >> 1) & 1) << 2));
    }
    auto issue = [&](int c) {
      char* img = smem + (c % NSLOT) * SLOT + pl * PC + rb * 128;
      const int t = c >> 2, k0 = (c & 3) * 64;
      const int kr = t ? op1.kr : op0.kr;
      const bf16* base = (t ? pb1 : pb0) + (kr ? k0 * NL + o0w : o0w * NL + k0);
#pragma unroll
      for (int i = 0; i < PPW; ++i)
        __builtin_amdgcn_global_load_lds((glb_t*)(base + (kr ? loff[1][i] : loff[0][i])), (lds_t*)(img + i * 1024),
                                         16, 0, DMA_POL);
    };
    if (SPLIT_DBG != 1) {
      issue(0);
      issue(1);  // nch >= 4
    }
    for (int c = 0; c < nchl; ++c) {
      if (c + 1 < nch) wait_vm<PPW>(); else wait_vm<0>();
      __builtin_amdgcn_s_barrier();  // chunk c landed (every producer); slot (c+2)%3 read by every consumer
      asm volatile("" ::: "memory");
      if (c + 2 < nch && SPLIT_DBG != 1) issue(c + 2);
    }
  } else {  // ---------------------------------------------------------------- consumer
    const int wm = wv >> 1, wn = wv & 1;
    const int code0 = J.a[0].kr | (J.b[0].kr << 1), code1 = J.a[1].kr | (J.b[1].kr << 1);
    const unsigned lbase = lds_off(smem);
    unsigned akc[4], bkc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      akc[s] = lbase + kc_addr(wm * 32, s, lane);
      bkc[s] = lbase + kc_addr(wn * 32, s, lane);
    }
    const unsigned akr = lbase + kr_addr(wm * 32, lane), bkr = lbase + kr_addr(wn * 32, lane);
    f32x16 acc = (f32x16){};
    if (st_on) ts[2] = stamp();
    for (int c = 0; c < nchl; ++c) {
      __builtin_amdgcn_s_barrier();  // chunk c landed; every consumer is done with chunk c-1
      asm volatile("" ::: "memory");
      if (st_on && c == 0) ts[3] = stamp();
      if (SPLIT_DBG == 2) continue;
      const unsigned sb = (c % NSLOT) * SLOT;
      switch ((c >> 2) ? code1 : code0) {
        case 0: chunk_mma<0, 0>(acc, sb, akr, bkr, akc, bkc); break;
        case 1: chunk_mma<1, 0>(acc, sb, akr, bkr, akc, bkc); break;
        case 2: chunk_mma<0, 1>(acc, sb, akr, bkr, akc, bkc); break;
        default: chunk_mma<1, 1>(acc, sb, akr, bkr, akc, bkc); break;
      }
      if (st_on && c == 0) ts[4] = stamp();
    }
    if (st_on) ts[5] = stamp();
    const int h = lane >> 5, cc = lane & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) ep[(wm * 32 + acc_row(r, h)) * EROW + wn * 32 + cc] = acc[r];
  }
  __syncthreads();  // the tile is in `ep`; every wave (producers too) takes one 8-element row piece
  __shared__ float dred[8];   // DOT: the 8 epilogue waves' partial dots
  if (SPLIT_DBG == 3 || !epi) {
    if (dotj && SPLIT_DBG != 3) __syncthreads();   // the one barrier the epilogue waves' dot sum takes
    return;
  }
  const float diag = J.diag, e1s = J.e1s, e2s = J.e2s;
  float ic = 1.f;
  if (need_c) ic = nbh <= 64 ? 1.f / (wave_max(mcv) * wave_max(mrv)) : inv_c(maxima, nbh);
  const float alpha = J.alpha * powc(ic, J.alpha_cpow);
  const float e1m = powc(ic, J.e1_cpow);
  auto edecode = [&](const f32x4 (&r)[2], int f32, float* v) {
    if (f32) {
      const f32x4 x = r[0], y = r[1];
      v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3]; v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
    } else {
      const bf16x8 hh = __builtin_bit_cast(bf16x8, r[0]), ll = __builtin_bit_cast(bf16x8, r[1]);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (float)hh[e] + (float)ll[e];
    }
  };
  {
    const int row = m0 + lr, col = n0 + lc;
    const bool dg = row >= col && row < col + 8;  // the piece holds the diagonal element (row, row)
    float s[8], e1v[8], e2v[8], v[8];
    {
      const f32x4 x0 = *(const f32x4*)(ep + lr * EROW + lc), x1 = *(const f32x4*)(ep + lr * EROW + lc + 4);
      s[0] = x0[0]; s[1] = x0[1]; s[2] = x0[2]; s[3] = x0[3]; s[4] = x1[0]; s[5] = x1[1]; s[6] = x1[2]; s[7] = x1[3];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { s[e] *= alpha; e1v[e] = 0.f; e2v[e] = 0.f; }
    if (e1p) {
      edecode(e1raw, e1f, e1v);
#pragma unroll
      for (int e = 0; e < 8; ++e) e1v[e] *= e1m;
    }
    if (!dotj && e2p) edecode(e2raw, e2f, e2v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = s[e] + e1s * e1v[e] + e2s * e2v[e];
    if (dg) v[row - col] += diag;
    // write-through outputs: the launch-end L2 write-back would otherwise hold the next level's start
    // (forward chain 91.4 -> 85.5 us, backward 170.8 -> 169.1 us in graph replay; diagnostic variant 6
    // = plain stores for the A/B, scripts/dev/pinv_graph_stamps.py --ab 0,6)
    const bool wt = SPLIT_DBG != 6;
    if (J.c_f32) store_f8((float*)J.c, eoff, v, wt); else store_split8((bf16*)J.c, plane, eoff, v, wt);
    if (!dotj && J.cf) store_f8(J.cf, eoff, v, wt);
    if (J.c2) {
      float w[8];
      const float c2a = J.c2_alpha, c2e = J.c2_e1;
#pragma unroll
      for (int e = 0; e < 8; ++e) w[e] = c2a * s[e] + c2e * e1v[e];
      if (dg) w[row - col] += J.c2_diag;
      store_split8(J.c2, plane, eoff, w, wt);
    }
    if (J.c3) {
      float w[8];
      const float c3e = J.c3_e1;
#pragma unroll
      for (int e = 0; e < 8; ++e) w[e] = c3e * e1v[e];
      store_split8(J.c3, plane, eoff, w, wt);
    }
    if (dotj) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(v[e], dxv[e], d);
      d = wave_sum(d);
      if (lane == 0) dred[wv] = d;
      __syncthreads();   // every wave of the workgroup (the non-epilogue ones at their return)
      if (tid == 0)
        job_dot_part(J)[(size_t)head * 16 + tile] =
            ((dred[0] + dred[1]) + (dred[2] + dred[3])) + ((dred[4] + dred[5]) + (dred[6] + dred[7]));
    }
  }
  if (st_on && wv < 4) {
    ts[6] = stamp();
    ts[7] = rstamp();
    if (lane == 0) {
      unsigned long long* o = stamp_out + wv * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = ts[i];
    }
  }
}

// One launch = up to three independent jobs over all heads.  Grid: (16 * nbh, njobs);
// blockIdx.y is the job.
// AUX: the launch carries the A3 combine row (only the forward's last level; a separate
// instantiation, so the other levels' code is not touched by the combine's registers)
template <bool AUX, bool DOT = false>
__global__ __launch_bounds__(NTHREADS) void pinv_stage_kernel(SLaunch L) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (AUX && blockIdx.y == (unsigned)L.njobs) {
    // the A3 combine row: three 256-thread groups per workgroup, one item (head, 8 queries) each
    A3CombineLds* lds = (A3CombineLds*)smem;
    const int g = threadIdx.x >> 8, t = threadIdx.x & 255;
    const int item = blockIdx.x * (NTHREADS / 256) + g;
    const bool active = item < L.a3.nbh * 32;
    const int bh = active ? item >> 5 : 0, qy = item & 31;
    const A3CombineState st = a3_combine_phase1(L.a3, bh, qy, t, lds[g], active);
    __syncthreads();
    a3_combine_phase2(L.a3, bh, qy, t, lds[g], st, active);
    return;
  }
  const SJob& J = L.j[blockIdx.y];
  const int u = blockIdx.x;
  const int nbh = L.nbh;
  const int head = u % nbh, tile = u / nbh;
  if (J.kind == KIND_ABSSUMS) {
    if (u < 2 * nbh) abssums(L, head, tile, (float*)smem);
    if (L.zero_ctr && u == 0 && threadIdx.x < TEAM_CTR_WORDS) L.zero_ctr[threadIdx.x] = 0u;
    return;
  }
  const int dbg_ = L.dbg;
  if (SPLIT_DBG == 5) return;
  unsigned long long* so = L.stamps ? L.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 * 8 : nullptr;
  stage_tile<false, 16, DOT>(J, nbh, L.plane, L.maxima, head, tile, smem, so, dbg_,
                             DOT && (int)blockIdx.y == L.njobs - 1);
}

// ---------------------------------------------------------------------------
// Backward of Z_0 = X^T / c (c = max_i rowsum|X|_i * max_j colsum|X|_j) and of A2 = softmax.
// part: npart partial dots of sum_ij G0[i][j] X[j][i], written by the backward chain's last level
// (SJob.dotx: one per wave of every output tile).
// dX[i][j] = dXc[i][j] + G0[j][i]/c + sign(X_ij) (tie_c(i) dMc/nc + tie_r(j) dMr/nr),
// dc = -sum(G0 o Z0)/c = -T/c^2,  dMc = dc * maxr, dMr = dc * maxc  (max ties share the gradient);
// softmax != 0: out = X o (dX - rowsum(X o dX)) (the backward of A2 = softmax, X = A2), else out = dX.
// grid (nbh, 256 / APPLY_ROWS), block 256: APPLY_ROWS rows of one head, thread = column j.
constexpr int APPLY_ROWS = 4;   // 512 workgroups at nbh = 8 (16 rows: 128, half the CUs idle)
constexpr int APPLY_SUMS = 8;   // |X| sums per thread per kind in one burst (nbh <= 8); larger nbh loops
__global__ __launch_bounds__(256) void pinv_apply_bwd_kernel(const float* __restrict__ X, const float* __restrict__ sums,
                                                             const float* __restrict__ maxima, const bf16* __restrict__ G0,
                                                             long long plane, const float* __restrict__ part, int npart,
                                                             int nbh,
                                                             const float* __restrict__ dXc, int softmax,
                                                             float* __restrict__ out) {
  __shared__ float red[4][16];
  __shared__ float bc[4];
  constexpr int RB = APPLY_ROWS;
  const int bh = blockIdx.x, i0 = blockIdx.y * RB, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const size_t hb = (size_t)bh * MAT;
  // every load is issued up front (one memory round trip): G0[t][i0..i0+15] (the transpose term of
  // column t, 32 contiguous bytes per plane), X and dXc rows i0..i0+15 at column t, this block's
  // row sums and column sum, the per-head maxima (lane h), the |X| sums for the tie counts and the
  // partial dots (lane-strided, clamped, masked)
  static_assert(RB == 4 || RB == 8, "one 8- or 16-B piece per plane of G0's transposed row");
  float g0[RB], xv[RB], dx[RB];
  {
    const size_t o = hb + (size_t)t * NL + i0;
    if constexpr (RB == 8) {
      const bf16x8 h0 = *(const bf16x8*)(G0 + o), l0 = *(const bf16x8*)(G0 + plane + o);
#pragma unroll
      for (int e = 0; e < 8; ++e) g0[e] = (float)h0[e] + (float)l0[e];
    } else {
      const bf16x4 h0 = *(const bf16x4*)(G0 + o), l0 = *(const bf16x4*)(G0 + plane + o);
#pragma unroll
      for (int e = 0; e < 4; ++e) g0[e] = (float)h0[e] + (float)l0[e];
    }
  }
#pragma unroll
  for (int ii = 0; ii < RB; ++ii) {
    const size_t off = hb + (size_t)(i0 + ii) * NL + t;
    xv[ii] = X[off];
    dx[ii] = dXc[off];
  }
  const float* rs = sums + (size_t)bh * NL;
  const float* cs = sums + (size_t)(nbh + bh) * NL;
  const float csv = cs[t];
  float rsv[RB];
#pragma unroll
  for (int q = 0; q < RB / 4; ++q) {
    const f32x4 v = *(const f32x4*)(rs + i0 + 4 * q);
    rsv[4 * q] = v[0]; rsv[4 * q + 1] = v[1]; rsv[4 * q + 2] = v[2]; rsv[4 * q + 3] = v[3];
  }
  const int total = nbh * NL;
  float sc[APPLY_SUMS], sr[APPLY_SUMS];
#pragma unroll
  for (int u = 0; u < APPLY_SUMS; ++u) {
    const int e = min(t + 256 * u, total - 1);
    sc[u] = sums[e];
    sr[u] = sums[total + e];
  }
  const float mcl = lane < nbh ? maxima[lane] : -INFINITY, mrl = lane < nbh ? maxima[nbh + lane] : -INFINITY;
  float ps = t < npart ? part[t] : 0.f;
  // global maxima (nbh <= 64: one lane per head), tie counts, the fixed-order partial-dot sum
  float mc = wave_max(mcl), mr = wave_max(mrl);
  for (int h = 64; h < nbh; ++h) { mc = fmaxf(mc, maxima[h]); mr = fmaxf(mr, maxima[nbh + h]); }
  float nc = 0.f, nr = 0.f;
#pragma unroll
  for (int u = 0; u < APPLY_SUMS; ++u)
    if (t + 256 * u < total) { nc += sc[u] == mc; nr += sr[u] == mr; }
  for (int e = t + 256 * APPLY_SUMS; e < total; e += 256) { nc += sums[e] == mc; nr += sums[total + e] == mr; }
  for (int e = t + 256; e < npart; e += 256) ps += part[e];
  nc = wave_sum(nc); nr = wave_sum(nr); ps = wave_sum(ps);
  if (lane == 0) { red[wave][0] = nc; red[wave][1] = nr; red[wave][2] = ps; }
  __syncthreads();
  if (t == 0) {
    bc[0] = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
    bc[1] = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
    bc[2] = (red[0][2] + red[1][2]) + (red[2][2] + red[3][2]);
  }
  __syncthreads();
  const float c = mc * mr, ic = 1.f / c;
  const float dc = -bc[2] * ic * ic;
  const float dMc = dc * mr / bc[0], dMr = dc * mc / bc[1];
  const float tie_r = csv == mr ? dMr : 0.f;
#pragma unroll
  for (int ii = 0; ii < RB; ++ii) {
    const float sg = xv[ii] > 0.f ? 1.f : (xv[ii] < 0.f ? -1.f : 0.f);
    const float tie_c = rsv[ii] == mc ? dMc : 0.f;
    dx[ii] = dx[ii] + g0[ii] * ic + sg * (tie_c + tie_r);
  }
  if (!softmax) {
#pragma unroll
    for (int ii = 0; ii < RB; ++ii) out[hb + (size_t)(i0 + ii) * NL + t] = dx[ii];
    return;
  }
  __syncthreads();
#pragma unroll
  for (int ii = 0; ii < RB; ++ii) {
    const float d = wave_sum(xv[ii] * dx[ii]);
    if (lane == 0) red[wave][ii] = d;
  }
  __syncthreads();
#pragma unroll
  for (int ii = 0; ii < RB; ++ii) {
    const float rd = (red[0][ii] + red[1][ii]) + (red[2][ii] + red[3][ii]);
    out[hb + (size_t)(i0 + ii) * NL + t] = xv[ii] * (dx[ii] - rd);
  }
}

// ---------------------------------------------------------------------------
// The chain as levels of independent jobs (shared by the host launch path and the device-side
// persistent kernel, so both run the same products).
#define TM_HD __host__ __device__ inline

TM_HD SOp op(const void* p, int kr) { return SOp{(const bf16*)p, kr, 0}; }

TM_HD SJob product(SOp a, SOp b, void* c, float alpha, float diag = 0.f) {
  SJob j{};
  j.kind = KIND_PRODUCT;
  j.nterms = 1;
  j.a[0] = a; j.b[0] = b;
  j.c = c;
  j.alpha = alpha; j.diag = diag;
  return j;
}

// saved-buffer layout (floats); every slot is nbh*MAT floats
struct FwdLayout {
  long long mat;
  int iters;
  float* base;
  TM_HD float* zf() const { return base; }                                      // Z_iters fp32
  TM_HD bf16* z(int k) const { return (bf16*)(base + (long long)k * mat); }     // Z_k split, k = 1..iters
  TM_HD bf16* p(int k) const { return (bf16*)(base + (long long)(iters + 1 + k) * mat); }  // P_k, k = 0..iters-1
  TM_HD bf16* t3(int k) const { return (bf16*)(base + (long long)(2 * iters + 1 + k) * mat); }
  TM_HD bf16* t5(int k) const { return (bf16*)(base + (long long)(3 * iters + 1 + k) * mat); }
  TM_HD bf16* scratch(int i) const { return (bf16*)(base + (long long)(4 * iters + 1 + i) * mat); }
  TM_HD float* sums() const { return base + (long long)(4 * iters + 3) * mat; }
  TM_HD float* maxima(int nbh) const { return sums() + 2LL * nbh * NL; }
  // the persistent kernel's counters (forward set 0, backward set 1), 64-B aligned after the maxima
  TM_HD unsigned* team_ctr(int nbh, int set) const {
    const uintptr_t e = (uintptr_t)(maxima(nbh) + 2 * nbh);
    return (unsigned*)((e + 63) & ~(uintptr_t)63) + set * TEAM_SET_WORDS;
  }
};

TM_HD FwdLayout fwd_layout(float* saved, int nbh, int iters) {
  FwdLayout f;
  f.mat = (long long)nbh * MAT;
  f.iters = iters;
  f.base = saved;
  return f;
}

struct ChainArgs {
  const bf16* Xs;   // split X (= A2)
  float* saved;     // FwdLayout
  float* work;      // backward workspace (G, dT5, dZa, dP, dT3, dXc, partial dots)
  int nbh, iters;
  const float* X = nullptr;   // fp32 X: the backward's last level also writes the c-gradient dots
  float* part = nullptr;      //   (per-wave partials of sum G0 o X^T) when set
};

// forward levels after L1 (S = X X^T + the |X| sums): A_0, B_0, A_1, B_1, ..., A_{it-1}, B_{it-1}, F
TM_HD int fwd_levels(int iters) { return 2 * iters + 1; }
TM_HD int fwd_level_njobs(int iters, int lvl) {
  if (lvl == 2 * iters) return 1;
  const int k = lvl >> 1;
  return (lvl & 1) == 0 ? (k >= 1 ? 2 : 1) : (k + 1 < iters ? 2 : 1);
}
TM_HD SJob fwd_level_job(const ChainArgs& a, int lvl, int jn) {
  const FwdLayout F = fwd_layout(a.saved, a.nbh, a.iters);
  const int iters = a.iters;
  if (lvl == 2 * iters) {  // F: Z_iters = 0.25 Z_{iters-1} T5_{iters-1}  (split + fp32)
    SJob z = iters == 1 ? product(op(a.Xs, 1), op(F.t5(0), 1), F.z(1), 0.25f)
                        : product(op(F.z(iters - 1), 0), op(F.t5(iters - 1), 1), F.z(iters), 0.25f);
    if (iters == 1) z.alpha_cpow = 1;
    z.cf = F.zf();
    return z;
  }
  const int k = lvl >> 1;
  bf16* R = F.scratch((k + 1) & 1);
  if ((lvl & 1) == 0) {  // A_k: R = P P (T3 = R - 7P + 15I); Z_k = 0.25 Z_{k-1} T5_{k-1}
    if (jn == 0) {
      SJob r;
      if (k == 0) {  // P_0 = S / c: R = S S / c^2, T3 = R - 7 S/c + 15I, P_0 written as a side output
        r = product(op(F.scratch(0), 0), op(F.scratch(0), 1), R, 1.f);
        r.alpha_cpow = 2;
        r.e1 = F.scratch(0); r.e1_cpow = 1;
        r.c3 = F.p(0); r.c3_e1 = 1.f;
      } else {
        r = product(op(F.p(k), 0), op(F.p(k), 1), R, 1.f);
        r.e1 = F.p(k);
      }
      r.c2 = F.t3(k); r.c2_alpha = 1.f; r.c2_diag = 15.f; r.c2_e1 = -7.f;
      return r;
    }
    SJob z = k == 1 ? product(op(a.Xs, 1), op(F.t5(0), 1), F.z(1), 0.25f)           // Z_0 = X^T / c
                    : product(op(F.z(k - 1), 0), op(F.t5(k - 1), 1), F.z(k), 0.25f);
    if (k == 1) z.alpha_cpow = 1;
    return z;
  }
  // B_k: T5 = 13I - P T3; P_{k+1} = 3.25 P - 0.25 R T3
  if (jn == 0) return product(op(F.p(k), 0), op(F.t3(k), 1), F.t5(k), -1.f, 13.f);
  SJob p = product(op(R, 0), op(F.t3(k), 1), F.p(k + 1), -0.25f);
  p.e1 = F.p(k); p.e1s = 3.25f;
  return p;
}

// backward levels (the reference graph's adjoint), 4 per iteration, k = iters-1 .. 0
TM_HD int bwd_levels(int iters) { return 4 * iters; }
TM_HD int bwd_level_njobs(int iters, int lvl) { return (lvl & 3) == 2 ? 1 : 2; }
TM_HD SJob bwd_level_job(const ChainArgs& a, int lvl, int jn) {
  const FwdLayout F = fwd_layout(a.saved, a.nbh, a.iters);
  const long long mat = F.mat;
  float* work = a.work;
  bf16* G = (bf16*)work;
  bf16* dT5 = (bf16*)(work + mat);
  bf16* dZa = (bf16*)(work + 2 * mat);
  bf16* dP = (bf16*)(work + 3 * mat);
  bf16* dT3 = (bf16*)(work + 4 * mat);
  float* dXc = work + 5 * mat;
  const int k = a.iters - 1 - (lvl >> 2);
  switch (lvl & 3) {
    case 0:  // dT5 = 0.25 Z_k^T G ; dZa = 0.25 G T5_k^T
      if (jn == 0) {
        SJob j = k == 0 ? product(op(a.Xs, 0), op(G, 1), dT5, 0.25f)          // Z_0^T = X / c
                        : product(op(F.z(k), 1), op(G, 1), dT5, 0.25f);
        if (k == 0) j.alpha_cpow = 1;
        return j;
      }
      return product(op(G, 0), op(F.t5(k), 0), dZa, 0.25f);
    case 1:  // dP = -dT5 T3^T ; dT3 = -P^T dT5
      if (jn == 0) return product(op(dT5, 0), op(F.t3(k), 0), dP, -1.f);
      return product(op(F.p(k), 1), op(dT5, 1), dT3, -1.f);
    case 2: {  // dP += dT3 P^T + P^T dT3 - 7 dT3   (T3 = P P - 7P + 15I)
      SJob j = product(op(dT3, 0), op(F.p(k), 0), dP, 1.f);
      j.nterms = 2;
      j.a[1] = op(F.p(k), 1); j.b[1] = op(dT3, 1);
      j.e1 = dP; j.e1s = 1.f;
      j.e2 = dT3; j.e2s = -7.f;
      return j;
    }
    default:  // dX (+)= dP Z_k^T ; G = dZa + X^T dP
      if (jn == 0) {
        SJob j = k == 0 ? product(op(dP, 0), op(a.Xs, 1), dXc, 1.f)            // Z_0^T = X / c
                        : product(op(dP, 0), op(F.z(k), 0), dXc, 1.f);
        if (k == 0) j.alpha_cpow = 1;
        j.c_f32 = 1;
        if (k != a.iters - 1) { j.e1 = dXc; j.e1_f32 = 1; j.e1s = 1.f; }
        return j;
      }
      SJob g = product(op(a.Xs, 1), op(dP, 1), G, 1.f);
      g.e1 = dZa; g.e1s = 1.f;
      if (k == 0 && a.X) { g.e2 = a.X; g.cf = a.part; }   // G = G0: the c gradient's dot (DOT launch)
      return g;
  }
}

#ifdef TM_DIAG
// ---------------------------------------------------------------------------
// Persistent chain kernel: every level of the forward (after L1) or of the backward in ONE
// launch, instead of one launch per level (each launch boundary + ramp + first operand fetch
// from beyond L2 costs ~3-4 us of the ~6.5 us a level took).
//
// Teams by XCD: a workgroup reads its XCD (HW_REG_XCC_ID) and works only on the heads
// h = xcd (mod 8).  Every matrix of a head is then written and read by workgroups of ONE XCD
// within this launch, so the hand-off stays in that XCD's L2 (the L2 is the coherence point of
// its CUs): producers store plainly and drain (s_waitcnt vmcnt(0), barrier) before one
// device-scope atomic add on the team's done counter; consumers poll it with L1-bypassing loads
// and read every operand with L1-bypassing loads (LDS-DMA sc1, epilogue operands nt), so no
// stale L1 line is ever used and no L2 write-back / invalidate is needed between levels.  The
// operands written before this launch (X, the per-head maxima) come through the launch boundary.
//
// Work queue per team: a ticket counter hands out the team's tile-jobs in level order (level l
// has njobs(l) x 16 tiles x its heads); a workgroup waits, before its tile-job, until the done
// counter covers every tile-job of the earlier levels.  A ticket is only ever held by a running
// workgroup and waits only on lower tickets, so the queue cannot deadlock whatever subset of the
// grid is resident (another stream's kernels may hold CUs); every workgroup leaves once a
// ticket is past the last level, and the last one to leave zeroes the counters for the next call.
// A wait is bounded (~1 s): on expiry the error word is set and the workgroup leaves.
//
// Measured and rejected (diagnostic build only, variant 8): correct (test_pinv_split_gpu), but a
// level still takes ~6 us -- a tile is bound by its own operand fill (128 KB per term into one
// CU's LDS at ~31 B/clk: ~2 us, plus ~1.2 us to the first chunk and ~0.7 us of epilogue), and the
// counter hand-off between levels costs ~1.1 us, the same as a launch boundary in graph replay.
// Whole step in graph replay: 734 vs 758 slides/s with one launch per level
// (scripts/dev/team_stamps.py, scripts/dev/ab_split_variant.py).
struct TeamArgs {
  ChainArgs c;
  int dir;             // 0: forward levels, 1: backward levels
  long long plane;
  const float* maxima;
  unsigned* ctr;       // TEAM_SET_WORDS: per XCD [ticket, .., done @ +16], then the exit count and error word
  unsigned long long* stamps;   // diagnostic build: per ticket 40 u64 (stage stamps, then claim / ready / done / xcc / level)
};

constexpr int TEAM_GRID = 256;   // one workgroup per CU (113 KB of LDS each)
// diagnostic stamps: ticket t of XCD x at record x * 512 + t
TM_DEV unsigned t_global_base(int x, unsigned t) { return (unsigned)x * 512u + t; }

template <int POL>
__global__ __launch_bounds__(NTHREADS) void pinv_team_kernel(TeamArgs T) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  volatile unsigned* bc = (volatile unsigned*)(smem + STAGE_LDS + EPI_LDS);
  const int tid = threadIdx.x;
  const int x = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;   // HW_REG_XCC_ID
  const int nbh = T.c.nbh, iters = T.c.iters;
  const int nh = nbh > x ? (nbh - 1 - x) / TEAM_XCD + 1 : 0;       // heads x, x + 8, ... of this team
  unsigned* ticket = T.ctr + x * TEAM_STRIDE;
  unsigned* done = ticket + TEAM_STRIDE / 2;
  unsigned* exits = T.ctr + TEAM_XCD * TEAM_STRIDE;
  unsigned* err = exits + 1;
  const int nlev = T.dir == 0 ? fwd_levels(iters) : bwd_levels(iters);
  const unsigned per_job = 16u * (unsigned)nh;
  unsigned prefix = 0;   // tile-jobs of the levels before `lev`
  int lev = 0;
  while (nh > 0) {
#ifdef TM_DIAG
    const unsigned long long t_claim = T.stamps ? rstamp() : 0;
#endif
    if (tid == 0) bc[0] = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned t = __builtin_amdgcn_readfirstlane(bc[0]);
    while (lev < nlev) {
      const unsigned cnt = per_job * (T.dir == 0 ? fwd_level_njobs(iters, lev) : bwd_level_njobs(iters, lev));
      if (t < prefix + cnt) break;
      prefix += cnt;
      ++lev;
    }
    if (lev >= nlev) break;
    if (tid == 0) {   // every tile-job of the earlier levels done (relaxed L1-bypassing polls, bounded)
      unsigned polls = 0;
      while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < prefix) {
        __builtin_amdgcn_s_sleep(2);
        if (++polls > (1u << 24)) { __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
      }
    }
    __syncthreads();   // also: every wave has read bc[0]
    const unsigned r = t - prefix;
    const int jn = (int)(r / per_job), rem = (int)(r % per_job);
    const int head = x + TEAM_XCD * (rem >> 4), tile = rem & 15;
    const SJob J = T.dir == 0 ? fwd_level_job(T.c, lev, jn) : bwd_level_job(T.c, lev, jn);
    unsigned long long* so = nullptr;
#ifdef TM_DIAG
    const unsigned long long t_ready = T.stamps ? rstamp() : 0;
    if (T.stamps) so = T.stamps + (size_t)t_global_base(x, t) * 40;
#endif
    stage_tile<true, POL, true>(J, nbh, T.plane, T.maxima, head, tile, smem, so, 0,
                                T.dir == 1 && lev == nlev - 1 && jn == 1 && T.c.X != nullptr);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's tile stores have reached the L2
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef TM_DIAG
    if (so && tid == 0) {
      so[32] = t_claim; so[33] = t_ready; so[34] = rstamp(); so[35] = x; so[36] = lev; so[37] = jn; so[38] = tile;
    }
#endif
  }
  if (tid == 0) {
    const unsigned e = __hip_atomic_fetch_add(exits, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e == gridDim.x - 1) {   // the last workgroup out: nothing of this launch touches the counters any more
      for (int i = 0; i < TEAM_XCD; ++i) {
        __hip_atomic_store(T.ctr + i * TEAM_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(T.ctr + i * TEAM_STRIDE + TEAM_STRIDE / 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(exits, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
#endif  // TM_DIAG

// ---------------------------------------------------------------------------
// host side
struct Launcher {
  SLaunch L{};
  explicit Launcher(int nbh, long long plane, const float* maxima) {
    L.nbh = nbh; L.plane = plane; L.maxima = maxima;
#ifdef TM_DIAG
    L.dbg = g_split_dbg;
    L.stamps = g_split_stamps;
#endif
  }
  bool dot = false;   // the last job's e2 / cf carry the c-gradient dot (job_dotx / job_dot_part)
  void add(const SJob& j) { L.j[L.njobs++] = j; }
  int go(hipStream_t st) {
    dim3 grid(16 * L.nbh, L.njobs);
    if (L.a3.w) {   // one more row for the A3 combine: ceil(nbh * 32 / 3) <= 16 nbh items
      grid.y += 1;
      tm_allow_smem(pinv_stage_kernel<true>, STAGE_LDS + EPI_LDS);
      pinv_stage_kernel<true><<<grid, NTHREADS, STAGE_LDS + EPI_LDS, st>>>(L);
    } else if (dot) {   // the backward's last level: the c-gradient dot in its epilogue
      tm_allow_smem(pinv_stage_kernel<false, true>, STAGE_LDS + EPI_LDS);
      pinv_stage_kernel<false, true><<<grid, NTHREADS, STAGE_LDS + EPI_LDS, st>>>(L);
    } else {
      tm_allow_smem(pinv_stage_kernel<false>, STAGE_LDS + EPI_LDS);
      pinv_stage_kernel<false><<<grid, NTHREADS, STAGE_LDS + EPI_LDS, st>>>(L);
    }
    TM_CHECK_LAUNCH();
#ifdef TM_DIAG
    if (g_split_stamps) g_split_stamps += (size_t)grid.x * grid.y * 4 * 8;  // the next launch's stamps follow
#endif
    return 0;
  }
};

// the levels [0, nlev) of one direction: one launch per level (or, diagnostic build variant 8,
// the persistent kernel)
int run_levels(const ChainArgs& c, int dir, long long plane, const float* maxima, unsigned* ctr, hipStream_t st,
               const A3Combine* a3 = nullptr) {
#ifdef TM_DIAG
  if (g_split_dbg == 8 || g_split_dbg == 9) {   // 9: plain-policy DMA (timing probe only: L1 may be stale)
    TeamArgs T{c, dir, plane, maxima, ctr, g_split_stamps};
    auto kern = g_split_dbg == 8 ? pinv_team_kernel<16> : pinv_team_kernel<0>;
    tm_allow_smem(kern, STAGE_LDS + EPI_LDS + 64);
    kern<<<TEAM_GRID, NTHREADS, STAGE_LDS + EPI_LDS + 64, st>>>(T);
    TM_CHECK_LAUNCH();
    return 0;
  }
#else
  (void)ctr;
#endif
  const int nlev = dir == 0 ? fwd_levels(c.iters) : bwd_levels(c.iters);
  for (int lvl = 0; lvl < nlev; ++lvl) {
    Launcher l(c.nbh, plane, maxima);
    const int nj = dir == 0 ? fwd_level_njobs(c.iters, lvl) : bwd_level_njobs(c.iters, lvl);
    for (int j = 0; j < nj; ++j) l.add(dir == 0 ? fwd_level_job(c, lvl, j) : bwd_level_job(c, lvl, j));
    l.dot = dir == 1 && lvl == nlev - 1 && c.X != nullptr;
    if (a3 && dir == 0 && lvl == nlev - 1) l.L.a3 = *a3;   // the forward's last level: one 128-tile job
    if (int rc = l.go(st)) return rc;
  }
  return 0;
}

}  // namespace

extern "C" long long tm_pinv_split_saved_floats(int nbh, int iters) {
  // ... + the maxima, then the persistent kernel's two counter sets on 64-B lines
  return (4LL * iters + 3) * nbh * MAT + 2LL * nbh * NL + 2LL * nbh + 16 + TEAM_CTR_WORDS + 64;
}

// X: fp32 [nbh][256][256]; Xs: its split planes (tm_nys_sim2_softmax_split).  saved: see FwdLayout;
// Z_iters (fp32) sits at the start of `saved`.  Two launches: L1 (S = X X^T and the |X| sums /
// maxima, which couple all heads through c, and the zeroed team counters), then every other
// level in the persistent kernel.
int pinv_fwd_split(const float* X, const void* Xs, int nbh, int iters, float* saved, const A3Combine* a3,
                   void* stream);

extern "C" int tm_pinv_fwd_split(const float* X, const void* Xs, int nbh, int iters, float* saved, void* stream) {
  return pinv_fwd_split(X, Xs, nbh, iters, saved, nullptr, stream);
}

// as tm_pinv_fwd_split, and the A3 forward's partial combine (tm_nys_a3_fwd with w = null left the
// partials in a3_work: part_o [P][nbh][256][64] bf16 in an fp32-sized region, then part_m, part_l
// [P][nbh][256] fp32) runs beside the
// chain's last product: W and lse3 are written by the same launch that writes Z_iters.
extern "C" int tm_pinv_fwd_split_a3(const float* X, const void* Xs, int nbh, int iters, float* saved,
                                    const float* a3_work, int a3_parts, float* w, float* lse3, void* stream) {
  TM_REQUIRE(a3_work && w && lse3 && a3_parts >= 1, "pinv_fwd_split_a3: bad A3 args");
  const bf16* po = (const bf16*)a3_work;   // bf16 partial sums in the first half of their fp32-sized region
  const float* pm = a3_work + (size_t)a3_parts * nbh * NL * 64;
  const float* pl = pm + (size_t)a3_parts * nbh * NL;
  const A3Combine a3{po, pm, pl, a3_parts, nbh, w, lse3};
  return pinv_fwd_split(X, Xs, nbh, iters, saved, &a3, stream);
}

int pinv_fwd_split(const float* X, const void* Xs, int nbh, int iters, float* saved, const A3Combine* a3,
                   void* stream) {
  TM_REQUIRE(X && Xs && saved && nbh > 0 && iters >= 1, "pinv_fwd_split: bad args (iters >= 1)");
  TM_REQUIRE(((uintptr_t)Xs % 16) == 0 && ((uintptr_t)saved % 16) == 0, "pinv_fwd_split: 16-B aligned buffers");
  hipStream_t st = (hipStream_t)stream;
  const FwdLayout F = fwd_layout(saved, nbh, iters);
  const long long plane = F.mat;
  float* maxima = F.maxima(nbh);
  {  // L1: S = X X^T, |X| sums
    Launcher l(nbh, plane, nullptr);
    l.add(product(op(Xs, 0), op(Xs, 0), F.scratch(0), 1.f));
    SJob s{};
    s.kind = KIND_ABSSUMS;
    l.add(s);
    l.L.X = X; l.L.sums = F.sums(); l.L.maxima_out = maxima;
    l.L.zero_ctr = F.team_ctr(nbh, 0);   // both counter sets (forward, then backward)
    if (int rc = l.go(st)) return rc;
  }
  const ChainArgs c{(const bf16*)Xs, saved, nullptr, nbh, iters};
  return run_levels(c, 0, plane, maxima, F.team_ctr(nbh, 0), st, a3);
}

// workspace: G, dT5, dZa, dP, dT3 (split) + dX (fp32) + partial dots
extern "C" long long tm_pinv_bwd_split_workspace_floats(int nbh) {
  return 6LL * nbh * MAT + nbh * 16LL + 64;
}

// dZ: the gradient w.r.t. Z_iters as split planes, placed by the caller at the start of `work`
// (tm_bmm with c_split).  out: dL/dX (softmax == 0) or dL/d(sim2 logits) = softmax backward of
// A2 = X (softmax != 0), fp32.  `saved` is the forward's; its backward counter set is used (and
// left zeroed) by the persistent kernel.
extern "C" int tm_pinv_bwd_split(const float* X, const void* Xs, int nbh, int iters, const float* saved, float* work,
                                 int softmax, float* out, void* stream) {
  TM_REQUIRE(X && Xs && saved && work && out && nbh > 0 && iters >= 1, "pinv_bwd_split: bad args");
  hipStream_t st = (hipStream_t)stream;
  const FwdLayout F = fwd_layout((float*)saved, nbh, iters);
  const long long mat = F.mat, plane = mat;
  const float* maxima = F.maxima(nbh);
  bf16* G = (bf16*)work;
  float* dXc = work + 5 * mat;
  float* part = work + 6 * mat;
  ChainArgs c{(const bf16*)Xs, (float*)saved, work, nbh, iters};
  c.X = X;      // the last level writes G0 and the c gradient's per-wave dots sum G0 o X^T
  c.part = part;
  if (int rc = run_levels(c, 1, plane, maxima, F.team_ctr(nbh, 1), st)) return rc;
  // Z_0 = X^T / c: the transpose term, the max-tie terms and the softmax
  pinv_apply_bwd_kernel<<<dim3(nbh, NL / APPLY_ROWS), 256, 0, st>>>(X, F.sums(), maxima, G, plane, part, nbh * 16, nbh, dXc,
                                                        softmax, out);
  TM_CHECK_LAUNCH();
  return 0;
}

#ifdef TM_DIAG
extern "C" void tm_debug_set_split_variant(int v) { g_split_dbg = v; }
// diagnostic: per-wave stamps (8 x u64 per wave, 8 waves per workgroup) of every later stage launch; null: off
extern "C" void tm_debug_set_split_stamps(unsigned long long* buf) { g_split_stamps = buf; }
#endif

// fp32 -> split planes (hi at dst, lo at dst + count), count a multiple of 8
__global__ void split_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long count) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= count) return;
  float v[8];
  load_f8(x, i, v);
  store_split8(y, count, i, v);
}

extern "C" int tm_split_f32(const float* x, void* y, long long count, void* stream) {
  TM_REQUIRE(count % 8 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0, "split_f32: count % 8, alignment");
  if (count == 0) return 0;
  split_kernel<<<(unsigned)((count / 8 + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, (bf16*)y, count);
  TM_CHECK_LAUNCH();
  return 0;
}
