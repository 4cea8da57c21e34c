// Shared device helpers for the TransMIL HIP kernels (gfx950 / CDNA4 only).
//
// Element types: every kernel is instantiated for T = float ("parity" mode, f32
// MFMA: exact fmaf chains) and T = bf16 ("bench" mode, bf16 MFMA with fp32
// accumulation).  Softmax, LayerNorm statistics, the pseudo-inverse and the
// residual stream are always fp32.
//
// MFMA conventions (32x32 tiles, 64-lane waves):
//   A fragment  lane l: row r = l&31, k = 8*(l>>5) + j, j = 0..7   (8 consecutive k)
//   B fragment  lane l: col r = l&31, k = 8*(l>>5) + j
//   C/D         reg i : row = (i&3) + 8*(i>>2) + 4*(l>>5), col = l&31
// For bf16 one v_mfma_f32_32x32x16_bf16 consumes the 8-element fragments; for
// f32 eight v_mfma_f32_32x32x2_f32 do, instruction j taking element j (lane
// half h supplies k = 8h + j), so the same fragment loaders serve both types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

#define TM_DEV __device__ __forceinline__

// Ablation / diagnostic switches exist only in the TM_DIAG build (`make diag` ->
// libtransmil_hip_diag.so, loaded by scripts/microbench.py through TRANSMIL_HIP_LIB).  The product
// library has no process-global mutable state: every selector is the constant 0 (the default
// kernel), the alternative kernels are not compiled and no tm_debug_* symbol is exported.
#ifdef TM_DIAG
#define TM_DIAG_VAR(v) (v)
#else
#define TM_DIAG_VAR(v) 0
#endif

template <typename T> struct V8;
template <> struct V8<bf16> { typedef bf16x8 type; };
template <> struct V8<float> { typedef f32x8 type; };
template <typename T> using vec8 = typename V8<T>::type;

template <typename T> struct V4;
template <> struct V4<bf16> { typedef bf16x4 type; };
template <> struct V4<float> { typedef f32x4 type; };
template <typename T> using vec4 = typename V4<T>::type;

TM_DEV float to_f(float x) { return x; }
TM_DEV float to_f(bf16 x) { return (float)x; }
template <typename T> TM_DEV T from_f(float x);
template <> TM_DEV float from_f<float>(float x) { return x; }
template <> TM_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

// 8 consecutive elements (16 B for bf16, 2 x 16 B for f32).  p must be 16-B aligned.
template <typename T> TM_DEV vec8<T> load8(const T* p);
template <> TM_DEV bf16x8 load8<bf16>(const bf16* p) { return *(const bf16x8*)p; }
template <> TM_DEV f32x8 load8<float>(const float* p) {
  f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  return (f32x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
template <typename T> TM_DEV void store8(T* p, vec8<T> v);
template <> TM_DEV void store8<bf16>(bf16* p, bf16x8 v) { *(bf16x8*)p = v; }
template <> TM_DEV void store8<float>(float* p, f32x8 v) {
  *(f32x4*)p = (f32x4){v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = (f32x4){v[4], v[5], v[6], v[7]};
}
// 4 consecutive elements (8 B bf16 / 16 B f32)
template <typename T> TM_DEV vec4<T> load4(const T* p) { return *(const vec4<T>*)p; }
template <typename T> TM_DEV void store4(T* p, vec4<T> v) { *(vec4<T>*)p = v; }

// 8 consecutive floats -> vec8<T> (used when an fp32 tensor feeds a T MFMA)
template <typename T> TM_DEV vec8<T> cvt8(const float* p) {
  f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  vec8<T> r;
  r[0] = from_f<T>(a[0]); r[1] = from_f<T>(a[1]); r[2] = from_f<T>(a[2]); r[3] = from_f<T>(a[3]);
  r[4] = from_f<T>(b[0]); r[5] = from_f<T>(b[1]); r[6] = from_f<T>(b[2]); r[7] = from_f<T>(b[3]);
  return r;
}

// acc += A_frag * B_frag over one 16-deep k step
TM_DEV void mma16(f32x16& c, const bf16x8& a, const bf16x8& b) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
TM_DEV void mma16(f32x16& c, const f32x8& a, const f32x8& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], c, 0, 0, 0);
}

// Accumulator tile X (rows on registers) as the B operand of the next product
// that sums over X's rows: registers 8s..8s+7 form k-step s (s = 0, 1); element
// j of lane half h is row 16s + 8(j>>2) + 4h + (j&3) of X.  The A operand must
// supply the same k for element j (see acc_k_index()).
template <typename T> TM_DEV vec8<T> acc_as_operand(const f32x16& x, int s) {
  vec8<T> r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = from_f<T>(x[8 * s + j]);
  return r;
}
// row of X (0..31) that element j of lane half h carries in k-step s
TM_DEV int acc_k_index(int s, int h, int j) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }
// row of a C/D register
TM_DEV int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Raw buffer loads with hardware bounds: an offset at or past `bytes` returns zeros, so a masked
// (zero-padded) tile load is ONE unconditional instruction (no exec-mask branch around it, 32-bit
// offsets).  Resource word 3 = 0x00020000 for gfx9 (raw, 32-bit data format).
TM_DEV __amdgpu_buffer_rsrc_t tm_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
TM_DEV f32x4 tm_bload4(__amdgpu_buffer_rsrc_t r, unsigned off_bytes) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, 0));
}
constexpr unsigned TM_OOB = 0xFFFFFFF0u;   // an offset past every resource

TM_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
TM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Whole-wave max / sum on DPP lane moves (no LDS round trip per step, as __shfl_xor's ds_bpermute
// takes): quads, half rows, rows of 16, then the row broadcasts 15 / 31 fold the four rows into lane
// 63, read back as a wave-uniform value.  A fixed combination order (deterministic sums).
template <int CTRL, int ROW_MASK = 0xf>
TM_DEV float dpp_mov(float old, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                               CTRL, ROW_MASK, 0xf, false));
}
TM_DEV float wave_max_dpp(float v) {
  const float ninf = -INFINITY;
  v = fmaxf(v, dpp_mov<0xB1>(ninf, v));         // quad_perm [1, 0, 3, 2]
  v = fmaxf(v, dpp_mov<0x4E>(ninf, v));         // quad_perm [2, 3, 0, 1]
  v = fmaxf(v, dpp_mov<0x141>(ninf, v));        // row_half_mirror
  v = fmaxf(v, dpp_mov<0x140>(ninf, v));        // row_mirror: every lane holds its row's max
  v = fmaxf(v, dpp_mov<0x142, 0xa>(ninf, v));   // row_bcast:15 into rows 1, 3
  v = fmaxf(v, dpp_mov<0x143, 0xc>(ninf, v));   // row_bcast:31 into rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
TM_DEV float wave_sum_dpp(float v) {
  v += dpp_mov<0xB1>(0.f, v);
  v += dpp_mov<0x4E>(0.f, v);
  v += dpp_mov<0x141>(0.f, v);
  v += dpp_mov<0x140>(0.f, v);
  v += dpp_mov<0x142, 0xa>(0.f, v);
  v += dpp_mov<0x143, 0xc>(0.f, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

TM_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
TM_DEV float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Counter-based dropout hash: uniform in [0,1) from (seed, row, col).
TM_DEV uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
TM_DEV float dropout_u01(uint64_t seed, uint32_t row, uint32_t col) {
  uint32_t h = mix32((uint32_t)seed ^ mix32(row * 0x9E3779B1u + (uint32_t)(seed >> 32)));
  h = mix32(h ^ (col * 0x7FEB352Du));
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

TM_DEV uint64_t effective_seed(uint64_t seed, const uint64_t* seed_ptr) {
  return seed_ptr ? (*seed_ptr) * 0x9E3779B97F4A7C15ull + seed : seed;
}

// Error plumbing shared by every C entry point.
const char* tm_set_error(const char* msg);
#define TM_CHECK_LAUNCH()                                                   \
  do {                                                                      \
    hipError_t e__ = hipGetLastError();                                     \
    if (e__ != hipSuccess) { tm_set_error(hipGetErrorString(e__)); return 2; } \
  } while (0)
#define TM_REQUIRE(cond, msg)                                               \
  do { if (!(cond)) { tm_set_error(msg); return 1; } } while (0)

enum { TM_F32 = 0, TM_BF16 = 1 };

// Compute units of the current device (hipDeviceAttributeMultiprocessorCount), for grid sizing
// only (never for results' layout): a read-only per-device cache, so schedules follow the part
// the library runs on instead of assuming 256 CUs.
inline int tm_cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  static int cache[64];   // benign race: every writer stores the same device constant
  int v = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
  if (v <= 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    __atomic_store_n(&cache[dev], c, __ATOMIC_RELAXED);
    v = c;
  }
  return v;
}

// Opt a kernel into > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU).
template <typename K>
inline void tm_allow_smem(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
