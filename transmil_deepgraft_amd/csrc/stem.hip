// ResNet-50 stem of the C5 encoder in one pass (code/models/ResNet.py:240-245: conv1 7x7/2 pad 3,
// 3 -> 64 channels, bn1, relu, maxpool 3x3/2 pad 1), eval mode with the BatchNorm folded into the
// convolution: out = maxpool(relu(conv(x, w) + b)), bf16 in, channels-last bf16 out.  The library
// path (MIOpen convolution, then tm_bias_relu_maxpool) writes and re-reads the 112 x 112 x 64
// convolution output (1.6 MB per tile) and runs the 3-channel convolution at ~130 TF/s; here the
// convolution output never leaves the workgroup.
//
// One workgroup = an 8 x 8 block of pooled outputs of one tile.  It needs the 17 x 17 convolution
// outputs under those windows (conv rows 2P-1 .. 2P+15), i.e. 39 x 39 input pixels, which it
// stages in LDS as [row][col][4] bf16 (the three channels + a zero), 40 columns per row, read from
// any (n, c, h, w) element strides (NCHW tiles need no channels-last copy first).  The
// convolution is an implicit GEMM on v_mfma_f32_32x32x16_bf16: M = the 289 conv pixels (10 tiles
// of 32), N = 64 channels (2 tiles), K = 7 kernel rows x (8 columns x 4 channels) = 224, column 7
// and channel 3 carrying zero weights.  For a kernel row ky, the 32 k values of one conv pixel are
// 8 consecutive LDS pixels of input row 2r + ky starting at column 2c, so a lane's 8-element A
// fragment (k = 16 s + 8 h .. + 7 = 2 pixels x 4 channels) is one aligned 16-B LDS read.  The
// packed weights ([64][224], built once at fold time) sit in LDS at a padded row stride.  After the
// k loop the accumulators get + bias and ReLU, are rounded to bf16 and stored over the staging
// area as the 289 x 64 conv tile; each thread then takes the 3 x 3 max of one pooled pixel's 16
// channels over the conv pixels inside the image.
#include "common.h"

namespace {

constexpr int SP = 8;                      // pooled rows / cols per workgroup
constexpr int SCV = 2 * SP + 1;            // conv rows / cols under them: 17
constexpr int SNPIX = SCV * SCV;           // 289
constexpr int SMT = (SNPIX + 31) / 32;     // 10 M tiles
constexpr int SIR = 2 * SCV + 5;           // 39 input rows
constexpr int SIC = 40;                    // input columns in LDS (+ the zero-weight tap column 7)
constexpr int SK = 224;                    // 7 x 8 x 4
constexpr int SWROW = 232;                 // LDS row stride of the packed weights (elements)
constexpr int SOROW = 72;                  // LDS row stride of the conv tile (elements)
constexpr int SIMG_BYTES = SIR * SIC * 8;                  // 12480
constexpr int SW_BYTES = 64 * SWROW * 2;                   // 29696
constexpr int SOUT_BYTES = SNPIX * SOROW * 2;              // 41616
constexpr int SLDS = (SIMG_BYTES + SW_BYTES) > SOUT_BYTES ? SIMG_BYTES + SW_BYTES : SOUT_BYTES;
constexpr int STHREADS = 256;

#ifdef TM_DIAG
// diagnostics: per-workgroup clock stamps of wave 0 ([block][8]: realtime start, shader clock at
// start, staged, k loop done, conv tile stored, pool stores issued, realtime end), first 4096 blocks
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

template <bool STAMP = false>
__global__ __launch_bounds__(STHREADS) void stem_conv_pool_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wp,
                                                                  const bf16* __restrict__ bias, bf16* __restrict__ out,
                                                                  int H, int W, long long sn, long long sc,
                                                                  long long sh, long long sw, int CH, int CW, int PH,
                                                                  int PW, int nbr, int nbc) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[SLDS];
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  stem_stamp<STAMP>(ts, 0, true);
  stem_stamp<STAMP>(ts, 1);
  bf16* img = (bf16*)lds;                                   // [SIR][SIC][4]
  bf16* wl = (bf16*)(lds + SIMG_BYTES);                     // [64][SWROW]
  bf16* cv = (bf16*)lds;                                    // [SNPIX][SOROW], after the k loop
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 5, l32 = lane & 31;
  const int bc = blockIdx.x % nbc, br = (blockIdx.x / nbc) % nbr;
  const long long n = blockIdx.x / (nbc * nbr);
  const int P0 = br * SP, Q0 = bc * SP;                     // first pooled row / col
  const int cr0 = 2 * P0 - 1, cc0 = 2 * Q0 - 1;             // first conv row / col
  const int ir0 = 2 * cr0 - 3, ic0 = 2 * cc0 - 3;           // first input row / col

  // every global load of the staging goes out before the first LDS store (one latency, not one
  // per loop trip): packed weights (64 rows x 28 pieces of 16 B) and the input window, zero
  // outside the image (the convolution's zero padding)
  constexpr int WPIECES = 64 * (SK / 8), WTRIPS = (WPIECES + STHREADS - 1) / STHREADS;
  constexpr int IPIX = SIR * SIC, ITRIPS = (IPIX + STHREADS - 1) / STHREADS;
  bf16x8 wv8[WTRIPS];
#pragma unroll
  for (int t = 0; t < WTRIPS; ++t) {
    const int i = tid + t * STHREADS;
    if (i < WPIECES) wv8[t] = *(const bf16x8*)(wp + (i / (SK / 8)) * SK + (i % (SK / 8)) * 8);
  }
  // each channel value lands in its own register (zero-extended 16-bit load) and every load is
  // unconditional (an out-of-image pixel reads the tile's first element and is masked at the LDS
  // store): no per-trip wait before packing
  const unsigned short* xn = (const unsigned short*)x + n * sn;
  unsigned int iv[ITRIPS][3];
  bool iok[ITRIPS];
#pragma unroll
  for (int t = 0; t < ITRIPS; ++t) {
    const int i = tid + t * STHREADS;
    const int r = i / SIC, c = i % SIC;
    const int gh = ir0 + r, gw = ic0 + c;
    iok[t] = i < IPIX && gh >= 0 && gh < H && gw >= 0 && gw < W;
    const long long off = iok[t] ? gh * sh + gw * sw : 0;
    iv[t][0] = xn[off];
    iv[t][1] = xn[off + sc];
    iv[t][2] = xn[off + 2 * sc];
  }
#pragma unroll
  for (int t = 0; t < WTRIPS; ++t) {
    const int i = tid + t * STHREADS;
    if (i < WPIECES) *(bf16x8*)(wl + (i / (SK / 8)) * SWROW + (i % (SK / 8)) * 8) = wv8[t];
  }
#pragma unroll
  for (int t = 0; t < ITRIPS; ++t) {
    const int i = tid + t * STHREADS;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = iok[t] ? (u32x2){iv[t][0] | (iv[t][1] << 16), iv[t][2]} : (u32x2){0u, 0u};
    if (i < IPIX) *(u32x2*)(img + i * 4) = v;
  }
  // the lane's 32 bias values: output channel 32 u + 8 k + 4 g + e sits in acc[u][4 k + e]
  float bv[2][16];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) bv[u][i] = (float)bias[32 * u + acc_row(i, g)];
  __syncthreads();
  stem_stamp<STAMP>(ts, 2);

  // implicit GEMM, channels on the MFMA rows (A = weights) and conv pixels on its columns (B = the
  // input patches), so a lane ends with 4 consecutive channels per register quad of ONE pixel:
  // wave wv owns the pixel tiles wv, wv + 4, wv + 8 (< SMT) and both channel tiles
  f32x16 acc[3][2];
  int abase[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    acc[j][0] = (f32x16){};
    acc[j][1] = (f32x16){};
    int m = (wv + 4 * j) * 32 + l32;
    m = m < SNPIX ? m : SNPIX - 1;                          // padding columns: any in-range pixel
    const int lr = m / SCV, lc = m % SCV;
    abase[j] = ((2 * lr) * SIC + 2 * lc) * 4;
  }
  const int nt = wv + 8 < SMT ? 3 : 2;                      // wave-uniform
#pragma unroll
  for (int s = 0; s < SK / 16; ++s) {
    const int ky = s >> 1, kx0 = 4 * (s & 1) + 2 * g;
    const bf16x8 w0 = *(const bf16x8*)(wl + l32 * SWROW + 16 * s + 8 * g);
    const bf16x8 w1 = *(const bf16x8*)(wl + (32 + l32) * SWROW + 16 * s + 8 * g);
    const int koff = (ky * SIC + kx0) * 4;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j < nt) {
        const bf16x8 a = *(const bf16x8*)(img + abase[j] + koff);
        mma16(acc[j][0], w0, a);
        mma16(acc[j][1], w1, a);
      }
    }
  }
  __syncthreads();                                          // img / weights dead: cv overlays them
  stem_stamp<STAMP>(ts, 3);

  // + bias, ReLU, bf16 -> the conv tile in LDS: per register quad one 8-B store of 4 channels
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int m = (wv + 4 * j) * 32 + l32;
    if (j < nt && m < SNPIX) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (bf16)fmaxf(acc[j][u][4 * k + e] + bv[u][4 * k + e], 0.f);
          *(bf16x4*)(cv + m * SOROW + 32 * u + 8 * k + 4 * g) = o;
        }
    }
  }
  __syncthreads();
  stem_stamp<STAMP>(ts, 4);

  // 3 x 3 / 2 max pool: thread = (pooled pixel, 16 channels).  Conv pixels outside the image are
  // skipped (max_pool2d's -inf padding); every value is a ReLU output >= 0, so the max of the bf16
  // bit patterns as unsigned integers is the max of the values (no converts)
  const int p = tid >> 2, cg = (tid & 3) * 16;
  const int lpr = p / SP, lpc = p % SP;
  const int pr = P0 + lpr, pc = Q0 + lpc;
  if (pr < PH && pc < PW) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 lo[2] = {}, hi[2] = {};                           // the low / high bf16 of each dword
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int cr = 2 * pr - 1 + t / 3, cc = 2 * pc - 1 + t % 3;
      const unsigned keep = cr >= 0 && cr < CH && cc >= 0 && cc < CW ? 0xFFFFFFFFu : 0u;
      const int m = (2 * lpr + t / 3) * SCV + 2 * lpc + t % 3;   // always inside the tile
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const u32x4 u = *(const u32x4*)(cv + m * SOROW + cg + 8 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned v = u[e] & keep;                  // 0 (the max's identity here) off the image
          lo[h][e] = max(lo[h][e], v << 16);
          hi[h][e] = max(hi[h][e], v & 0xFFFF0000u);
        }
      }
    }
    u32x4 o0, o1;
#pragma unroll
    for (int e = 0; e < 4; ++e) { o0[e] = hi[0][e] | (lo[0][e] >> 16); o1[e] = hi[1][e] | (lo[1][e] >> 16); }
    bf16* q = out + ((n * PH + pr) * PW + pc) * 64 + cg;
    *(u32x4*)q = o0;
    *(u32x4*)(q + 8) = o1;
  }
#ifdef TM_DIAG
  if constexpr (STAMP) {
    stem_stamp<STAMP>(ts, 5);
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
  const int CH = (H - 1) / 2 + 1, CW = (W - 1) / 2 + 1;    // conv 7x7 / 2, pad 3
  const int PH = (CH - 1) / 2 + 1, PW = (CW - 1) / 2 + 1;  // pool 3x3 / 2, pad 1
  const int nbr = (PH + SP - 1) / SP, nbc = (PW + SP - 1) / SP;
  const long long blocks = (long long)N * nbr * nbc;
  TM_REQUIRE(blocks < (1ll << 31), "stem_conv_pool: too many tiles");
  if (TM_DIAG_VAR(g_stem_variant) == 1)
    stem_conv_pool_kernel<true><<<(unsigned)blocks, STHREADS, 0, (hipStream_t)stream>>>(
        (const bf16*)x, (const bf16*)wp, (const bf16*)bias, (bf16*)out, H, W, sn, sc, sh, sw, CH, CW, PH, PW, nbr, nbc);
  else
    stem_conv_pool_kernel<false><<<(unsigned)blocks, STHREADS, 0, (hipStream_t)stream>>>(
        (const bf16*)x, (const bf16*)wp, (const bf16*)bias, (bf16*)out, H, W, sn, sc, sh, sw, CH, CW, PH, PW, nbr, nbc);
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
