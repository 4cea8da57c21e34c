// The A3 forward's partial combine (SURVEY.md App. A eq. 5-8: W = softmax(q~ k^T) v over key
// splits, flash-decode style), as a device routine shared by its own launch (a3_combine_v2_kernel,
// nystrom.hip) and by the last launch of the split pseudo-inverse chain (pinv_split.hip), whose
// idle CUs run it beside the chain's final product.
//
// One item = (head bh, 8 landmark queries qy*8..+7) over 256 threads t: thread (query, 4 d) of
// one of two halves that take the even / odd partials (every load of a burst issued first); the
// odd half's running (max, sum, 4 outputs) go through LDS to the even half, which merges them in a
// fixed order (deterministic) and writes W[bh][q][d] and lse3[bh][q].
#pragma once
#include "common.h"

struct A3Combine {
  const bf16* part_o;    // [P][nbh][256][64]  sum_keys exp(s - m) v  (bf16; merged in fp32)
  const float* part_m;   // [P][nbh][256]      m
  const float* part_l;   // [P][nbh][256]      sum_keys exp(s - m)
  int P, nbh;
  float* w;              // [nbh][256][64]
  float* lse3;           // [nbh][256]
};

// LDS per item: 128 x (16 + 4 + 4) bytes
struct A3CombineLds {
  f32x4 xo[128];
  float xm[128], xl[128];
};

struct A3CombineState {
  float M, L;
  f32x4 acc;
};

// phase 1: this thread's half of the partials; the odd half parks its state in LDS
TM_DEV A3CombineState a3_combine_phase1(const A3Combine& c, int bh, int qy, int t, A3CombineLds& lds, bool active) {
  constexpr int U = 16;   // partials per thread per burst
  const int item = t & 127, half = t >> 7;
  const int qi = qy * 8 + (item >> 4), d4 = (item & 15) * 4;
  const size_t q0 = (size_t)bh * 256 + qi, pstride = (size_t)c.nbh * 256;
  A3CombineState s{-INFINITY, 0.f, (f32x4){0.f, 0.f, 0.f, 0.f}};
  if (active) {
    for (int p0 = half; p0 < c.P; p0 += 2 * U) {
      float mv[U], lv[U];
      f32x4 ov[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t pidx = (size_t)min(p0 + 2 * u, c.P - 1) * pstride + q0;
        mv[u] = c.part_m[pidx];
        lv[u] = c.part_l[pidx];
        const bf16x4 b = *(const bf16x4*)(c.part_o + pidx * 64 + d4);
        ov[u] = (f32x4){(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
      }
      float mb = s.M;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (p0 + 2 * u < c.P) mb = fmaxf(mb, mv[u]);
      const float cc = __expf(s.M - mb);    // M = -inf on the first burst: 0
      s.L *= cc;
      s.acc *= cc;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (p0 + 2 * u < c.P) {
          const float sc = __expf(mv[u] - mb);
          s.L += lv[u] * sc;
          s.acc += ov[u] * sc;
        }
      s.M = mb;
    }
    if (half) { lds.xo[item] = s.acc; lds.xm[item] = s.M; lds.xl[item] = s.L; }
  }
  return s;
}

// phase 2 (after a workgroup barrier): the even half merges and writes
TM_DEV void a3_combine_phase2(const A3Combine& c, int bh, int qy, int t, const A3CombineLds& lds,
                              const A3CombineState& s, bool active) {
  const int item = t & 127, half = t >> 7;
  if (!active || half) return;
  const int qi = qy * 8 + (item >> 4), d4 = (item & 15) * 4;
  const size_t q0 = (size_t)bh * 256 + qi;
  const float Mo = lds.xm[item], Mt = fmaxf(s.M, Mo);
  const float ca = s.M == -INFINITY ? 0.f : __expf(s.M - Mt), cb = Mo == -INFINITY ? 0.f : __expf(Mo - Mt);
  const float Lt = s.L * ca + lds.xl[item] * cb;
  const f32x4 at = s.acc * ca + lds.xo[item] * cb;
  *(f32x4*)(c.w + q0 * 64 + d4) = at / Lt;
  if (d4 == 0) c.lse3[q0] = Mt + __logf(Lt);
}
