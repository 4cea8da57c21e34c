// ResNet-50 stem of the C5 encoder in one pass (code/models/ResNet.py:240-245: conv1 7x7/2 pad 3,
// 3 -> 64 channels, bn1, relu, maxpool 3x3/2 pad 1), eval mode with the BatchNorm folded into the
// convolution: out = maxpool(relu(conv(x, w) + b)), bf16 in, channels-last bf16 out.  The library
// path (MIOpen convolution, then tm_bias_relu_maxpool) writes and re-reads the 112 x 112 x 64
// convolution output (1.6 MB per tile) and runs the 3-channel convolution at ~130 TF/s; here the
// convolution output never leaves the workgroup.
//
// Region = an 8 x 7 block of pooled outputs of one tile (224 x 224: 7 x 8 regions per tile).  It
// needs the 17 x 15 convolution outputs under those windows (conv rows 2P-1 .. 2P+15), i.e. 39 x 35
// input pixels, staged in LDS as [row][col][4] bf16 (the three channels + a zero), 36 columns per
// row, read from any (n, c, h, w) element strides (NCHW tiles need no channels-last copy first).
// The convolution is an implicit GEMM on v_mfma_f32_32x32x16_bf16 with the 64 output channels on
// the MFMA rows (A = the packed weights, 2 tiles) and the 255 conv pixels on its columns (B, 8
// tiles of 32: two per wave), K = 7 kernel rows x (8 columns x 4 channels) = 224, column 7 and
// channel 3 carrying zero weights.  For a kernel row ky the 32 k values of one conv pixel are 8
// consecutive LDS pixels of input row 2r + ky from column 2c, so a lane's 8-element fragment
// (k = 16 s + 8 h .. + 7 = 2 pixels x 4 channels) is one aligned 16-B LDS read.  A lane ends with 4
// consecutive channels of one pixel per register quad: + bias, ReLU, one bf16 rounding and one 8-B
// LDS store each, into the 255 x 64 conv tile (over the staging area); each thread then takes the
// 3 x 3 max of one pooled pixel's 16 channels over the conv pixels inside the image.
//
// Persistent: one workgroup per CU pair slot walks regions blockIdx.x, + gridDim.x, ...; the packed
// weights ([64][224], built once at fold time) are staged in LDS once per workgroup, and the next
// region's input pixels are fetched into registers while the current region runs its k loop,
// epilogue and pool (the staging latency was the largest phase of a one-region-per-workgroup form:
// 0.73 ms per 1024 tiles, stamps scripts/dev/stem_stamps.py).
#include "common.h"
#include <algorithm>

namespace {

constexpr int SPR = 8, SPC = 7;                       // pooled rows / cols per region
constexpr int SCR = 2 * SPR + 1, SCC = 2 * SPC + 1;   // conv rows / cols under them: 17 x 15
constexpr int SNPIX = SCR * SCC;                      // 255
constexpr int SMT = (SNPIX + 31) / 32;                // 8 pixel tiles
constexpr int SIR = 2 * SCR + 5;                      // 39 input rows
constexpr int SIC = 2 * SCC + 6;                      // 36 input columns (35 + the zero-weight tap)
constexpr int SK = 224;                               // 7 x 8 x 4
constexpr int SWROW = 232;                            // LDS row stride of the packed weights (elements)
constexpr int SOROW = 72;                             // LDS row stride of the conv tile (elements)
constexpr int SW_BYTES = 64 * SWROW * 2;              // 29696
constexpr int SIMG_BYTES = SIR * SIC * 8;             // 11232
constexpr int SOUT_BYTES = SNPIX * SOROW * 2;         // 36720
constexpr int SBUF = SIMG_BYTES > SOUT_BYTES ? SIMG_BYTES : SOUT_BYTES;
constexpr int SLDS = SW_BYTES + SBUF;                 // 66416: two workgroups per CU
constexpr int STHREADS = 256;
constexpr int IPIX = SIR * SIC, ITRIPS = (IPIX + STHREADS - 1) / STHREADS;
static_assert(SMT == 8, "two pixel tiles per wave");

#ifdef TM_DIAG
// diagnostics: per-workgroup clock stamps of wave 0 ([block][8]: realtime start, shader clock at
// start, first region staged, its k loop done, its conv tile stored, its pool stores issued,
// realtime end of the workgroup)
__device__ unsigned long long g_stem_stamps[4096 * 8];
int g_stem_variant = 0;
#endif
template <bool ON>
TM_DEV void stem_stamp(unsigned long long (&ts)[8], int slot, bool real = false) {
  if constexpr (ON) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    if (real) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    else asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    ts[slot] = t;
  }
}

struct StemArgs {
  const bf16* x; const bf16* wp; const bf16* bias; bf16* out;
  long long sn;
  int H, W, sc, sh, sw;             // element strides inside one tile (< 2^31)
  unsigned tile_bytes;              // one tile's extent: the buffer resource of its loads
  int CH, CW, PH, PW, nbr, nbc;
  int nregions;
};

template <bool STAMP = false>
__global__ __launch_bounds__(STHREADS, 2) void stem_conv_pool_kernel(StemArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  stem_stamp<STAMP>(ts, 0, true);
  stem_stamp<STAMP>(ts, 1);
  bf16* wl = (bf16*)lds;                                    // [64][SWROW], for the whole walk
  bf16* img = (bf16*)(lds + SW_BYTES);                      // [SIR][SIC][4]
  bf16* cv = img;                                           // [SNPIX][SOROW], after the k loop
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 5, l32 = lane & 31;
  int r = blockIdx.x;
  if (r >= a.nregions) return;                              // (the grid never exceeds the regions)

  // packed weights -> LDS once (64 rows x 28 pieces of 16 B)
  constexpr int WPIECES = 64 * (SK / 8), WTRIPS = (WPIECES + STHREADS - 1) / STHREADS;
#pragma unroll
  for (int t = 0; t < WTRIPS; ++t) {
    const int i = tid + t * STHREADS;
    if (i < WPIECES) *(bf16x8*)(wl + (i / (SK / 8)) * SWROW + (i % (SK / 8)) * 8) =
        *(const bf16x8*)(a.wp + (i / (SK / 8)) * SK + (i % (SK / 8)) * 8);
  }
  // the lane's 32 bias values: output channel 32 u + 8 k + 4 g + e sits in acc[.][u][4 k + e]
  float bv[2][16];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) bv[u][i] = (float)a.bias[32 * u + acc_row(i, g)];

  // a region's input window in registers: each channel value in its own register, every load a
  // raw buffer load whose out-of-image offsets point past the resource (the hardware returns 0: the
  // convolution's zero padding, no branch, no mask)
  unsigned int iv[ITRIPS][3];
  const int ppt = a.nbr * a.nbc;                            // regions per tile
  auto fetch = [&](int rr) {
    const int n = rr / ppt, rem = rr - n * ppt;
    const int br = rem / a.nbc, bc = rem - br * a.nbc;
    const __amdgpu_buffer_rsrc_t rs = tm_rsrc(a.x + (long long)n * a.sn, a.tile_bytes);
    const int ir0 = 2 * (2 * br * SPR - 1) - 3, ic0 = 2 * (2 * bc * SPC - 1) - 3;
#pragma unroll
    for (int t = 0; t < ITRIPS; ++t) {
      const int i = tid + t * STHREADS;
      const int gh = ir0 + i / SIC, gw = ic0 + i % SIC;
      // branch-free: bitwise predicate (no short-circuit control flow) and an arithmetic select
      const unsigned bad = (unsigned)(i >= IPIX) | (unsigned)((unsigned)gh >= (unsigned)a.H) |
                           (unsigned)((unsigned)gw >= (unsigned)a.W);
      const unsigned mask = 0u - bad;                       // all ones off the image
      const unsigned o = (unsigned)(gh * a.sh + gw * a.sw) * 2u;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        iv[t][c] = __builtin_amdgcn_raw_buffer_load_b16(rs, ((o + (unsigned)(c * a.sc) * 2u) & ~mask) | (TM_OOB & mask),
                                                        0, 0);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int t = 0; t < ITRIPS; ++t) {
      const int i = tid + t * STHREADS;
      typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
      if (i < IPIX) *(u32x2*)(img + i * 4) = (u32x2){iv[t][0] | (iv[t][1] << 16), iv[t][2]};
    }
  };

  // this lane's two conv pixels (B columns) and their LDS patch bases
  int abase[2];
  int mpix[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    mpix[j] = (wv + 4 * j) * 32 + l32;
    const int m = mpix[j] < SNPIX ? mpix[j] : SNPIX - 1;    // the padding column: any pixel
    abase[j] = ((2 * (m / SCC)) * SIC + 2 * (m % SCC)) * 4;
  }

  fetch(r);
  stage();
  __syncthreads();
  stem_stamp<STAMP>(ts, 2);
  bool first = true;
  for (; r < a.nregions; r += gridDim.x) {
    const int rn = r + gridDim.x;
    if (rn < a.nregions) fetch(rn);                         // in flight during this region
    const int n = r / ppt, rem = r - n * ppt;
    const int br = rem / a.nbc, bc = rem - br * a.nbc;
    const int P0 = br * SPR, Q0 = bc * SPC;

    f32x16 acc[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) { acc[j][0] = (f32x16){}; acc[j][1] = (f32x16){}; }
#pragma unroll
    for (int s = 0; s < SK / 16; ++s) {
      const int ky = s >> 1, kx0 = 4 * (s & 1) + 2 * g;
      const bf16x8 w0 = *(const bf16x8*)(wl + l32 * SWROW + 16 * s + 8 * g);
      const bf16x8 w1 = *(const bf16x8*)(wl + (32 + l32) * SWROW + 16 * s + 8 * g);
      const int koff = (ky * SIC + kx0) * 4;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 b = *(const bf16x8*)(img + abase[j] + koff);
        mma16(acc[j][0], w0, b);
        mma16(acc[j][1], w1, b);
      }
    }
    __syncthreads();                                        // img dead: cv overlays it
    if (first) stem_stamp<STAMP>(ts, 3);

    // + bias, ReLU, bf16 -> the conv tile: per register quad one 8-B store of 4 channels
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (mpix[j] < SNPIX) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (bf16)fmaxf(acc[j][u][4 * k + e] + bv[u][4 * k + e], 0.f);
            *(bf16x4*)(cv + mpix[j] * SOROW + 32 * u + 8 * k + 4 * g) = o;
          }
      }
    }
    __syncthreads();
    if (first) stem_stamp<STAMP>(ts, 4);

    // 3 x 3 / 2 max pool: thread = (pooled pixel, 16 channels).  Conv pixels outside the image
    // are skipped (max_pool2d's -inf padding); every value is a ReLU output >= 0, so the max of the
    // bf16 bit patterns as unsigned integers is the max of the values (no converts)
    const int p = tid >> 2, cg = (tid & 3) * 16;
    const int lpr = p / SPC, lpc = p % SPC;
    const int pr = P0 + lpr, pc = Q0 + lpc;
    if (p < SPR * SPC && pr < a.PH && pc < a.PW) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      u32x4 lo[2] = {}, hi[2] = {};                         // the low / high bf16 of each dword
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int cr = 2 * pr - 1 + t / 3, cc = 2 * pc - 1 + t % 3;
        const unsigned keep = cr >= 0 && cr < a.CH && cc >= 0 && cc < a.CW ? 0xFFFFFFFFu : 0u;
        const int m = (2 * lpr + t / 3) * SCC + 2 * lpc + t % 3;   // always inside the tile
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u32x4 u = *(const u32x4*)(cv + m * SOROW + cg + 8 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const unsigned v = u[e] & keep;                 // 0 (the max's identity here) off the image
            lo[h][e] = max(lo[h][e], v << 16);
            hi[h][e] = max(hi[h][e], v & 0xFFFF0000u);
          }
        }
      }
      u32x4 o0, o1;
#pragma unroll
      for (int e = 0; e < 4; ++e) { o0[e] = hi[0][e] | (lo[0][e] >> 16); o1[e] = hi[1][e] | (lo[1][e] >> 16); }
      bf16* q = a.out + (((long long)n * a.PH + pr) * a.PW + pc) * 64 + cg;
      *(u32x4*)q = o0;
      *(u32x4*)(q + 8) = o1;
    }
    __syncthreads();                                        // cv dead: the next region's pixels
    if (first) stem_stamp<STAMP>(ts, 5);
    first = false;
    if (rn < a.nregions) stage();
    __syncthreads();
  }
#ifdef TM_DIAG
  if constexpr (STAMP) {
    stem_stamp<STAMP>(ts, 6, true);
    if (tid < 7 && blockIdx.x < 4096) {
      unsigned long long v = 0;
#pragma unroll
      for (int k = 0; k < 7; ++k) v = tid == k ? ts[k] : v;
      g_stem_stamps[blockIdx.x * 8 + tid] = v;
    }
  }
#endif
}

}  // namespace

extern "C" int tm_stem_conv_pool(const void* x, const void* wp, const void* bias, void* out, int N, int H, int W,
                                 long long sn, long long sc, long long sh, long long sw, void* stream) {
  TM_REQUIRE(x && wp && bias && out && N > 0 && H > 0 && W > 0 && sn > 0 && sc > 0 && sh > 0 && sw > 0,
             "stem_conv_pool: bad args");
  TM_REQUIRE(((uintptr_t)wp % 16) == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)x % 2) == 0,
             "stem_conv_pool: aligned buffers (weights / output 16 B)");
  const long long extent = 2 * sc + (long long)(H - 1) * sh + (long long)(W - 1) * sw + 1;   // elements
  TM_REQUIRE(extent * 2 < (1ll << 31) - 16, "stem_conv_pool: one tile must span < 2 GiB");
  StemArgs a;
  a.x = (const bf16*)x; a.wp = (const bf16*)wp; a.bias = (const bf16*)bias; a.out = (bf16*)out;
  a.H = H; a.W = W; a.sn = sn; a.sc = (int)sc; a.sh = (int)sh; a.sw = (int)sw;
  a.tile_bytes = (unsigned)(extent * 2);
  a.CH = (H - 1) / 2 + 1; a.CW = (W - 1) / 2 + 1;            // conv 7x7 / 2, pad 3
  a.PH = (a.CH - 1) / 2 + 1; a.PW = (a.CW - 1) / 2 + 1;      // pool 3x3 / 2, pad 1
  a.nbr = (a.PH + SPR - 1) / SPR; a.nbc = (a.PW + SPC - 1) / SPC;
  const long long nreg = (long long)N * a.nbr * a.nbc;
  TM_REQUIRE(nreg < (1ll << 31), "stem_conv_pool: too many tiles");
  a.nregions = (int)nreg;
  const int grid = (int)std::min<long long>(nreg, 2LL * tm_cu_count());
  if (TM_DIAG_VAR(g_stem_variant) == 1) {
    tm_allow_smem(stem_conv_pool_kernel<true>, SLDS);
    stem_conv_pool_kernel<true><<<(unsigned)grid, STHREADS, SLDS, (hipStream_t)stream>>>(a);
  } else {
    tm_allow_smem(stem_conv_pool_kernel<false>, SLDS);
    stem_conv_pool_kernel<false><<<(unsigned)grid, STHREADS, SLDS, (hipStream_t)stream>>>(a);
  }
  TM_CHECK_LAUNCH();
  return 0;
}

#ifdef TM_DIAG
extern "C" void tm_debug_set_stem_variant(int v) { g_stem_variant = v; }
extern "C" int tm_debug_stem_stamps(unsigned long long* host, int count) {
  TM_REQUIRE(count > 0 && count <= 4096 * 8, "stem_stamps: bad count");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stem_stamps), count * sizeof(unsigned long long)) != hipSuccess) {
    tm_set_error("stem_stamps: copy");
    return 2;
  }
  return 0;
}
#endif
