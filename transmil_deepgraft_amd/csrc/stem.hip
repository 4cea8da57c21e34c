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
constexpr int SRED_BYTES = 2 * 4 * 64 * 4;            // MODE 1: the 4 row groups' (sum, count) per channel
static_assert(SMT == 8, "two pixel tiles per wave");

// MODE 0: eval, folded bias.  MODE 1: train-mode statistics of the conv output (bf16-rounded, as a
// materialised conv output would be): per workgroup a fixed-order (count, mean, M2) over the conv
// pixels its regions own (rows 2P .. 2P+15, cols 2Q .. 2Q+13: each pixel once), no pooled output.
// MODE 2: train-mode BatchNorm apply: each conv value bf16(relu(bf16(conv) * scale + shift)) (the
// arithmetic of tm_bn_apply on the rounded conv output), then the pool.

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
  const float* scale; const float* shift;   // MODE 2: train-mode BatchNorm (batch statistics)
  double* part;                             // MODE 1: [grid][64][3] (count, mean, M2) per workgroup
  long long sn;
  int H, W, sc, sh, sw;             // element strides inside one tile (< 2^31)
  unsigned tile_bytes;              // one tile's extent: the buffer resource of its loads
  int CH, CW, PH, PW, nbr, nbc;
  int nregions;
};

template <int MODE, bool STAMP = false>
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
  // the lane's 32 bias (MODE 0) / scale + shift (MODE 2) values: output channel 32 u + 8 k + 4 g + e
  // sits in acc[.][u][4 k + e]
  float bv[2][16], sv[2][16];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * u + acc_row(i, g);
      bv[u][i] = MODE == 0 ? (float)a.bias[c] : MODE == 2 ? a.scale[c] : 0.f;
      sv[u][i] = MODE == 2 ? a.shift[c] : 0.f;
    }
  // MODE 1: the workgroup's running (count, mean, M2) of channel tid (threads 0..63), fp64
  double wn = 0.0, wmean = 0.0, wm2 = 0.0;
  float* red = (float*)(lds + SW_BYTES + SBUF);             // MODE 1 scratch [2][4][64]

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
            for (int e = 0; e < 4; ++e) {
              const float v = acc[j][u][4 * k + e];
              if constexpr (MODE == 0) o[e] = (bf16)fmaxf(v + bv[u][4 * k + e], 0.f);
              else if constexpr (MODE == 1) o[e] = (bf16)v;
              else o[e] = (bf16)fmaxf(fmaf((float)(bf16)v, bv[u][4 * k + e], sv[u][4 * k + e]), 0.f);
            }
            *(bf16x4*)(cv + mpix[j] * SOROW + 32 * u + 8 * k + 4 * g) = o;
          }
      }
    }
    __syncthreads();
    if (first) stem_stamp<STAMP>(ts, 4);

    if constexpr (MODE == 1) {
      // this region's pixels: local rows 1 .. 16, cols 1 .. 14 inside the image; thread = (channel,
      // row group q: rows 1 + q, 5 + q, ..): sum and count, then the region mean, then M2 about it
      const int c = tid & 63, q = tid >> 6;
      const int cr0 = 2 * P0 - 1, cc0 = 2 * Q0 - 1;
      const int lrh = min(2 * SPR, a.CH - 1 - cr0), lch = min(2 * SPC, a.CW - 1 - cc0);
      float sum = 0.f;
      int cnt = 0;
      for (int lr = 1 + q; lr <= lrh; lr += 4)
        for (int lc = 1; lc <= lch; ++lc) { sum += (float)cv[(lr * SCC + lc) * SOROW + c]; ++cnt; }
      red[q * 64 + c] = sum;
      red[256 + q * 64 + c] = (float)cnt;
      __syncthreads();
      float rs = 0.f, rc = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) { rs += red[k * 64 + c]; rc += red[256 + k * 64 + c]; }
      const float rmean = rs / rc;
      float m2 = 0.f;
      for (int lr = 1 + q; lr <= lrh; lr += 4)
        for (int lc = 1; lc <= lch; ++lc) {
          const float d = (float)cv[(lr * SCC + lc) * SOROW + c] - rmean;
          m2 = fmaf(d, d, m2);
        }
      __syncthreads();                                      // every thread has read red's sums
      red[q * 64 + c] = m2;
      __syncthreads();
      if (q == 0) {
        const double rm2 = (double)red[c] + (double)red[64 + c] + (double)red[128 + c] + (double)red[192 + c];
        const double n = wn + (double)rc, delta = (double)rmean - wmean;     // Chan et al. merge
        wmean += delta * (double)rc / n;
        wm2 += rm2 + delta * delta * wn * (double)rc / n;
        wn = n;
      }
    } else {
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
    }
    __syncthreads();                                        // cv dead: the next region's pixels
    if (first) stem_stamp<STAMP>(ts, 5);
    first = false;
    if (rn < a.nregions) stage();
    __syncthreads();
  }
  if constexpr (MODE == 1) {
    if (tid < 64) {
      double* pp = a.part + ((size_t)blockIdx.x * 64 + tid) * 3;
      pp[0] = wn;
      pp[1] = wmean;
      pp[2] = wm2;
    }
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

// the statistics' combine: one thread per channel merges the workgroups' (count, mean, M2) in
// workgroup order (fixed: deterministic), then nn.BatchNorm2d's train-mode outputs -- scale / shift
// with the biased variance, running statistics with the unbiased one and the momentum
__global__ __launch_bounds__(64) void stem_stats_final_kernel(const double* __restrict__ part, int nparts,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* running_mean,
                                                             float* running_var, float momentum, float eps,
                                                             float* __restrict__ scale, float* __restrict__ shift) {
  const int c = threadIdx.x;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int b = 0; b < nparts; ++b) {
    const double* pp = part + ((size_t)b * 64 + c) * 3;
    const double nb = pp[0];
    if (nb <= 0.0) continue;
    const double tot = n + nb, delta = pp[1] - mean;
    mean += delta * nb / tot;
    m2 += pp[2] + delta * delta * n * nb / tot;
    n = tot;
  }
  const double var = n > 0.0 ? m2 / n : 0.0;
  const double sc = (double)gamma[c] / sqrt(var + (double)eps);
  scale[c] = (float)sc;
  shift[c] = (float)((double)beta[c] - mean * sc);
  if (running_mean) running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
  if (running_var)
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * (n > 1.0 ? var * n / (n - 1.0) : var));
}

int stem_setup(StemArgs& a, const void* x, const void* wp, int N, int H, int W, long long sn, long long sc,
               long long sh, long long sw, int* grid) {
  TM_REQUIRE(x && wp && N > 0 && H > 0 && W > 0 && sn > 0 && sc > 0 && sh > 0 && sw > 0, "stem: bad args");
  TM_REQUIRE(((uintptr_t)wp % 16) == 0 && ((uintptr_t)x % 2) == 0, "stem: aligned buffers (weights 16 B)");
  const long long extent = 2 * sc + (long long)(H - 1) * sh + (long long)(W - 1) * sw + 1;   // elements
  TM_REQUIRE(extent * 2 < (1ll << 31) - 16, "stem: one tile must span < 2 GiB");
  a = StemArgs{};
  a.x = (const bf16*)x; a.wp = (const bf16*)wp;
  a.H = H; a.W = W; a.sn = sn; a.sc = (int)sc; a.sh = (int)sh; a.sw = (int)sw;
  a.tile_bytes = (unsigned)(extent * 2);
  a.CH = (H - 1) / 2 + 1; a.CW = (W - 1) / 2 + 1;            // conv 7x7 / 2, pad 3
  a.PH = (a.CH - 1) / 2 + 1; a.PW = (a.CW - 1) / 2 + 1;      // pool 3x3 / 2, pad 1
  a.nbr = (a.PH + SPR - 1) / SPR; a.nbc = (a.PW + SPC - 1) / SPC;
  const long long nreg = (long long)N * a.nbr * a.nbc;
  TM_REQUIRE(nreg < (1ll << 31), "stem: too many tiles");
  a.nregions = (int)nreg;
  *grid = (int)std::min<long long>(nreg, 2LL * tm_cu_count());
  return 0;
}

template <int MODE>
int stem_launch(const StemArgs& a, int grid, void* stream) {
  if (TM_DIAG_VAR(g_stem_variant) == 1) {
    tm_allow_smem(stem_conv_pool_kernel<MODE, true>, SLDS + SRED_BYTES);
    stem_conv_pool_kernel<MODE, true><<<(unsigned)grid, STHREADS, SLDS + SRED_BYTES, (hipStream_t)stream>>>(a);
  } else {
    tm_allow_smem(stem_conv_pool_kernel<MODE, false>, SLDS + SRED_BYTES);
    stem_conv_pool_kernel<MODE, false><<<(unsigned)grid, STHREADS, SLDS + SRED_BYTES, (hipStream_t)stream>>>(a);
  }
  TM_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int tm_stem_conv_pool(const void* x, const void* wp, const void* bias, void* out, int N, int H, int W,
                                 long long sn, long long sc, long long sh, long long sw, void* stream) {
  StemArgs a;
  int grid = 0;
  if (int rc = stem_setup(a, x, wp, N, H, W, sn, sc, sh, sw, &grid)) return rc;
  TM_REQUIRE(bias && out && ((uintptr_t)out % 16) == 0, "stem_conv_pool: bias / 16-B aligned output");
  a.bias = (const bf16*)bias; a.out = (bf16*)out;
  return stem_launch<0>(a, grid, stream);
}

extern "C" long long tm_stem_bn_stats_workspace(void) { return 2LL * tm_cu_count() * 64 * 3; }

extern "C" int tm_stem_bn_stats(const void* x, const void* wp, int N, int H, int W, long long sn, long long sc,
                                long long sh, long long sw, const float* gamma, const float* beta,
                                float* running_mean, float* running_var, float momentum, float eps, float* scale,
                                float* shift, double* workspace, long long ws_doubles, void* stream) {
  StemArgs a;
  int grid = 0;
  if (int rc = stem_setup(a, x, wp, N, H, W, sn, sc, sh, sw, &grid)) return rc;
  TM_REQUIRE(gamma && beta && scale && shift && workspace, "stem_bn_stats: bad args");
  TM_REQUIRE(ws_doubles >= (long long)grid * 64 * 3, "stem_bn_stats: workspace too small");
  a.part = workspace;
  if (int rc = stem_launch<1>(a, grid, stream)) return rc;
  stem_stats_final_kernel<<<1, 64, 0, (hipStream_t)stream>>>(workspace, grid, gamma, beta, running_mean, running_var,
                                                             momentum, eps, scale, shift);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_stem_conv_pool_bn(const void* x, const void* wp, const float* scale, const float* shift, void* out,
                                    int N, int H, int W, long long sn, long long sc, long long sh, long long sw,
                                    void* stream) {
  StemArgs a;
  int grid = 0;
  if (int rc = stem_setup(a, x, wp, N, H, W, sn, sc, sh, sw, &grid)) return rc;
  TM_REQUIRE(scale && shift && out && ((uintptr_t)out % 16) == 0, "stem_conv_pool_bn: scale / shift / output");
  a.scale = scale; a.shift = shift; a.out = (bf16*)out;
  return stem_launch<2>(a, grid, stream);
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
