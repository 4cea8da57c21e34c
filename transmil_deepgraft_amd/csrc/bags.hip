// Feature-bag sampling on HBM-resident bags (code/datasets/feature_dataloader.py:335-431):
// one launch gathers every output row of a batch from the store slab [total_rows, F]:
//
//   dst[r][:] = src[i0[r]][:]                                   (plain draw; bit-exact copy)
//   dst[r][:] = (src[i0[r]][:] * wa[r]) + (src[i1[r]][:] * wb[r])  (mixup blend rows, :305-330;
//                                                                 two rounded products, one add,
//                                                                 as torch evaluates it)
//   dst[r][:] = 0                                               (i0[r] < 0: the zero padding, :397-398)
//
// The index vectors are drawn on the host with the reference's own RNG calls (torch.randperm /
// torch.rand / numpy choice), so the rows are those of the reference; the kernel is the
// HBM-bound part: 16-B vector loads/stores, one wave per 256 columns of a row.
#include "common.h"
#include "../../include/transmil_hip.h"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) gather_rows_kernel(const T* __restrict__ src, int F,
                                                          const long long* __restrict__ i0,
                                                          const long long* __restrict__ i1,
                                                          const float* __restrict__ wa,
                                                          const float* __restrict__ wb, int nrows,
                                                          T* __restrict__ dst) {
  // two rounded products and one rounded add, as torch evaluates x*a + y*(1-a): no FMA contraction
#pragma clang fp contract(off)
  constexpr int VEC = 16 / sizeof(T);
  const int r = blockIdx.y;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) * VEC;
  if (r >= nrows || c >= F) return;
  T* d = dst + (size_t)r * F + c;
  const long long a = i0[r];
  const long long b = i1 ? i1[r] : -1;
  if (F % VEC == 0) {
    typedef T vt __attribute__((ext_vector_type(VEC)));
    vt out;
    if (a < 0) {
      for (int e = 0; e < VEC; ++e) out[e] = from_f<T>(0.f);
    } else if (b < 0) {
      out = *(const vt*)(src + (size_t)a * F + c);
    } else {
      const vt x = *(const vt*)(src + (size_t)a * F + c), y = *(const vt*)(src + (size_t)b * F + c);
      const float fa = wa[r], fb = wb[r];
      for (int e = 0; e < VEC; ++e) {
        const float p = to_f(x[e]) * fa, q = to_f(y[e]) * fb;
        out[e] = from_f<T>(p + q);
      }
    }
    *(vt*)d = out;
    return;
  }
  for (int e = 0; e < VEC && c + e < F; ++e) {
    float v = 0.f;
    if (a >= 0 && b < 0) {
      d[e] = src[(size_t)a * F + c + e];
      continue;
    }
    if (a >= 0) {
      const float p = to_f(src[(size_t)a * F + c + e]) * wa[r], q = to_f(src[(size_t)b * F + c + e]) * wb[r];
      v = p + q;
    }
    d[e] = from_f<T>(v);
  }
}

}  // namespace

extern "C" int tm_gather_rows(int dtype, const void* src, int F, const long long* i0, const long long* i1,
                              const float* wa, const float* wb, int nrows, void* dst, void* stream) {
  TM_REQUIRE(src && dst && i0 && F > 0 && nrows >= 0, "gather_rows: bad args");
  TM_REQUIRE(!i1 || (wa && wb), "gather_rows: blend rows need both weights");
  if (nrows == 0) return 0;
  TM_REQUIRE(nrows <= 65535, "gather_rows: at most 65535 rows per launch");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_F32) {
    const dim3 grid(((F + 3) / 4 + 255) / 256, nrows);
    gather_rows_kernel<float><<<grid, 256, 0, st>>>((const float*)src, F, i0, i1, wa, wb, nrows, (float*)dst);
  } else if (dtype == TM_BF16) {
    const dim3 grid(((F + 7) / 8 + 255) / 256, nrows);
    gather_rows_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)src, F, i0, i1, wa, wb, nrows, (bf16*)dst);
  } else {
    tm_set_error("gather_rows: dtype must be TM_F32 or TM_BF16");
    return 1;
  }
  TM_CHECK_LAUNCH();
  return 0;
}
