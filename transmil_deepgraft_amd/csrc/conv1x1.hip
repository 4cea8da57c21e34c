// C5 tile encoder: a 1x1 convolution over channels-last activations is a GEMM over their
// [rows = n*h*w, cin] matrix.  Runs it as a hipBLASLt GEMM whose epilogue adds the folded
// conv+BN bias, the Bottleneck's residual (beta = 1 on the C operand) and applies the ReLU
// (code/models/ResNet.py:95-117: conv3 -> bn3 -> out + identity -> ReLU), so the block output is
// written once instead of GEMM store + a separate add/ReLU pass re-reading it (the add/ReLU pass
// was 19 % of the C5 eval kernel time at HBM speed, profiles/r04_c5_kernel_summary.txt).
//
// Column-major view (hipBLASLt): D^T [cout x rows] = W [cout x cin] . X^T [cin x rows], i.e.
// A = W stored [cout][cin] (col-major cin x cout, op T), B = X stored [rows][cin] (col-major
// cin x rows, op N), C = residual and D = y stored [rows][cout] (col-major cout x rows); the
// bias vector has one entry per D row (cout).  Plans (layouts + the heuristic's candidates and the
// chosen algorithm) are cached per shape, one hipBLASLt handle per device; matmul descriptors are
// cached per (shape, bias pointer) and never modified after creation; the workspace is the
// caller's (stream-ordered), so calls on two streams share no scratch.  tm_conv1x1 never waits on
// the device; tm_conv1x1_tune, called once per shape outside stream capture, times the candidates
// (the ABI's one synchronising entry point).  A library GEMM, not a hand-written kernel: the
// encoder is frozen and outside the NystromAttention / PPEG hot path.
#include "common.h"

#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>

constexpr long long kConv1x1MaxWorkspace = 32LL << 20;   // scratch the heuristic may ask of the caller

namespace {

constexpr int kMaxDev = 16;
constexpr long long kMaxRows = 1LL << 21;
constexpr int kCand = 32;  // heuristic candidates (tm_conv1x1_tune times them)

struct Plan {
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, cd = nullptr;
  hipblasLtMatmulHeuristicResult_t cand[kCand];
  int ncand = 0;
  int chosen = 0;          // index into cand: 0 (heuristic) until tm_conv1x1_tune picks the fastest
  bool tuned = false;
};

using Key = std::tuple<int, int, int, int, int, long long, int, int>;   // dev dtype relu bias res rows cin cout

std::mutex g_mu;
hipblasLtHandle_t g_handle[kMaxDev] = {};
std::map<Key, Plan> g_plans;
// immutable matmul descriptors (the bias pointer is an attribute): created once per (shape, bias)
std::map<std::pair<Key, const void*>, hipblasLtMatmulDesc_t> g_descs;

const char* lt_error(hipblasStatus_t s) {
  switch (s) {
    case HIPBLAS_STATUS_NOT_INITIALIZED: return "conv1x1: hipBLASLt not initialized";
    case HIPBLAS_STATUS_ALLOC_FAILED: return "conv1x1: hipBLASLt allocation failed";
    case HIPBLAS_STATUS_INVALID_VALUE: return "conv1x1: hipBLASLt invalid value";
    case HIPBLAS_STATUS_NOT_SUPPORTED: return "conv1x1: hipBLASLt: shape/epilogue not supported";
    case HIPBLAS_STATUS_EXECUTION_FAILED: return "conv1x1: hipBLASLt execution failed";
    default: return "conv1x1: hipBLASLt error";
  }
}

#define LT_CHECK(expr)                                                        \
  do {                                                                        \
    hipblasStatus_t s__ = (expr);                                             \
    if (s__ != HIPBLAS_STATUS_SUCCESS) { tm_set_error(lt_error(s__)); return 3; } \
  } while (0)

int handle_of(int dev, hipblasLtHandle_t* out) {
  if (!g_handle[dev]) LT_CHECK(hipblasLtCreate(&g_handle[dev]));
  *out = g_handle[dev];
  return 0;
}

int make_desc(int dtype, int relu, const void* bias, hipblasLtMatmulDesc_t* out) {
  const hipDataType t = dtype == TM_BF16 ? HIP_R_16BF : HIP_R_32F;
  hipblasLtMatmulDesc_t d = nullptr;
  LT_CHECK(hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t opA = HIPBLAS_OP_T, opB = HIPBLAS_OP_N;
  hipblasStatus_t s = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA));
  if (s == HIPBLAS_STATUS_SUCCESS)
    s = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB));
  const hipblasLtEpilogue_t epi = bias ? (relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS)
                                       : (relu ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT);
  if (s == HIPBLAS_STATUS_SUCCESS)
    s = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  if (bias && s == HIPBLAS_STATUS_SUCCESS) {
    const int32_t bt = (int32_t)t;
    s = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    if (s == HIPBLAS_STATUS_SUCCESS)
      s = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
  }
  if (s != HIPBLAS_STATUS_SUCCESS) {
    hipblasLtMatmulDescDestroy(d);
    LT_CHECK(s);
  }
  *out = d;
  return 0;
}

// the plan of one row piece: layouts and the heuristic's candidates for workspaces <= ws_bytes
// (candidates are found once per shape with the largest workspace any caller offered so far; a call
// with a smaller workspace picks the first candidate that fits)
int plan_of(hipblasLtHandle_t h, const Key& key, int dtype, int relu, const void* bias, long long rows, int cin,
            int cout, Plan** out) {
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    Plan p;
    const hipDataType t = dtype == TM_BF16 ? HIP_R_16BF : HIP_R_32F;
    LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, t, (uint64_t)cin, (uint64_t)cout, (int64_t)cin));
    LT_CHECK(hipblasLtMatrixLayoutCreate(&p.b, t, (uint64_t)cin, (uint64_t)rows, (int64_t)cin));
    LT_CHECK(hipblasLtMatrixLayoutCreate(&p.cd, t, (uint64_t)cout, (uint64_t)rows, (int64_t)cout));
    hipblasLtMatmulDesc_t d = nullptr;
    if (int rc = make_desc(dtype, relu, bias, &d)) return rc;
    hipblasLtMatmulPreference_t pref = nullptr;
    hipblasStatus_t s = hipblasLtMatmulPreferenceCreate(&pref);
    const uint64_t wsb = kConv1x1MaxWorkspace;
    if (s == HIPBLAS_STATUS_SUCCESS)
      s = hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    int n = 0;
    if (s == HIPBLAS_STATUS_SUCCESS)
      s = hipblasLtMatmulAlgoGetHeuristic(h, d, p.a, p.b, p.cd, p.cd, pref, kCand, p.cand, &n);
    if (pref) hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatmulDescDestroy(d);
    LT_CHECK(s);
    if (n < 1) {
      tm_set_error("conv1x1: hipBLASLt found no algorithm for this shape/epilogue");
      return 3;
    }
    p.ncand = n;
    it = g_plans.emplace(key, p).first;
  }
  *out = &it->second;
  return 0;
}

int desc_of(const Key& key, int dtype, int relu, const void* bias, hipblasLtMatmulDesc_t* out) {
  auto k = std::make_pair(key, bias);
  auto it = g_descs.find(k);
  if (it == g_descs.end()) {
    if (g_descs.size() >= 4096) {   // bounded: a caller cycling through bias buffers
      for (auto& e : g_descs) hipblasLtMatmulDescDestroy(e.second);
      g_descs.clear();
    }
    hipblasLtMatmulDesc_t d = nullptr;
    if (int rc = make_desc(dtype, relu, bias, &d)) return rc;
    it = g_descs.emplace(k, d).first;
  }
  *out = it->second;
  return 0;
}

// the algorithm a call uses: the chosen candidate if its workspace fits, else the first that fits
const hipblasLtMatmulHeuristicResult_t* pick(const Plan& p, long long ws_bytes) {
  if (p.cand[p.chosen].state == HIPBLAS_STATUS_SUCCESS && (long long)p.cand[p.chosen].workspaceSize <= ws_bytes)
    return &p.cand[p.chosen];
  for (int i = 0; i < p.ncand; ++i)
    if (p.cand[i].state == HIPBLAS_STATUS_SUCCESS && (long long)p.cand[i].workspaceSize <= ws_bytes) return &p.cand[i];
  return nullptr;
}

struct Args {
  int dtype; const void* x; const void* w; const void* bias; const void* residual; void* y;
  long long rows; int cin, cout, relu; void* ws; long long ws_bytes;
};

int check(const Args& a, int* dev) {
  TM_REQUIRE(a.x && a.w && a.y && a.rows >= 0 && a.cin > 0 && a.cout > 0, "conv1x1: bad args");
  TM_REQUIRE(a.dtype == TM_BF16 || a.dtype == TM_F32, "conv1x1: dtype");
  TM_REQUIRE(a.residual != a.y, "conv1x1: residual must not alias the output");
  TM_REQUIRE(a.ws_bytes >= 0 && (a.ws || a.ws_bytes == 0), "conv1x1: workspace");
  if (hipGetDevice(dev) != hipSuccess || *dev < 0 || *dev >= kMaxDev) {
    tm_set_error("conv1x1: no current device");
    return 2;
  }
  return 0;
}

// run (tune == false) or time-and-choose (tune == true) every row piece of the call
int conv1x1(const Args& a, bool tune, hipStream_t st) {
  int dev = 0;
  if (int rc = check(a, &dev)) return rc;
  if (a.rows == 0) return 0;
  if (tune) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    TM_REQUIRE(hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone,
               "conv1x1_tune: not during stream capture (it waits on timing events)");
  }
  std::lock_guard<std::mutex> lock(g_mu);
  hipblasLtHandle_t h = nullptr;
  if (int rc = handle_of(dev, &h)) return rc;
  // row pieces of at most kMaxRows: one launch per piece keeps hipBLASLt's grid / index math in
  // the range it is tuned for (a whole 4096-tile bag is 12.8 M rows at layer 1)
  const size_t esz = a.dtype == TM_BF16 ? 2 : 4;
  const float alpha = 1.f, beta = a.residual ? 1.f : 0.f;
  for (long long r0 = 0; r0 < a.rows; r0 += kMaxRows) {
    const long long nr = a.rows - r0 < kMaxRows ? a.rows - r0 : kMaxRows;
    const Key key{dev, a.dtype, a.relu ? 1 : 0, a.bias ? 1 : 0, a.residual ? 1 : 0, nr, a.cin, a.cout};
    Plan* p = nullptr;
    if (int rc = plan_of(h, key, a.dtype, a.relu ? 1 : 0, a.bias, nr, a.cin, a.cout, &p)) return rc;
    hipblasLtMatmulDesc_t d = nullptr;
    if (int rc = desc_of(key, a.dtype, a.relu ? 1 : 0, a.bias, &d)) return rc;
    const char* xp = (const char*)a.x + (size_t)r0 * a.cin * esz;
    char* yp = (char*)a.y + (size_t)r0 * a.cout * esz;
    const char* rp = a.residual ? (const char*)a.residual + (size_t)r0 * a.cout * esz : yp;
    if (tune && !p->tuned) {
      // one warm-up + three timed runs of every candidate that fits the workspace, on the call's
      // own operands (y is rewritten by the caller's real call after); keep the fastest
      hipEvent_t e0, e1;
      if (hipEventCreate(&e0) != hipSuccess) { tm_set_error("conv1x1_tune: event"); return 2; }
      if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); tm_set_error("conv1x1_tune: event"); return 2; }
      float best = 3.4e38f;
      int bi = p->chosen;
      for (int i = 0; i < p->ncand; ++i) {
        const hipblasLtMatmulHeuristicResult_t& c = p->cand[i];
        if (c.state != HIPBLAS_STATUS_SUCCESS || (long long)c.workspaceSize > a.ws_bytes) continue;
        if (hipblasLtMatmul(h, d, &alpha, a.w, p->a, xp, p->b, &beta, rp, p->cd, yp, p->cd, &c.algo, a.ws,
                            c.workspaceSize, st) != HIPBLAS_STATUS_SUCCESS)
          continue;
        (void)hipEventRecord(e0, st);
        for (int k = 0; k < 3; ++k)
          hipblasLtMatmul(h, d, &alpha, a.w, p->a, xp, p->b, &beta, rp, p->cd, yp, p->cd, &c.algo, a.ws,
                          c.workspaceSize, st);
        (void)hipEventRecord(e1, st);
        float ms = 0.f;
        if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms < best) {
          best = ms;
          bi = i;
        }
      }
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      p->chosen = bi;
      p->tuned = true;
      continue;
    }
    if (tune) continue;
    const hipblasLtMatmulHeuristicResult_t* c = pick(*p, a.ws_bytes);
    if (!c) {
      tm_set_error("conv1x1: no hipBLASLt algorithm fits the workspace");
      return 3;
    }
    LT_CHECK(hipblasLtMatmul(h, d, &alpha, a.w, p->a, xp, p->b, &beta, rp, p->cd, yp, p->cd, &c->algo, a.ws,
                             c->workspaceSize, st));
  }
  return 0;
}

}  // namespace

// y[rows, cout] = act(x[rows, cin] . w[cout, cin]^T (+ bias[cout]) (+ residual[rows, cout])),
// act = ReLU when relu != 0; bias NULL = none (the train-mode path: BN applied afterwards).
// Row-major buffers (channels-last activations), dtype TM_BF16 or TM_F32 for all of x, w, bias,
// residual, y (fp32 accumulation); residual may be NULL and must not alias y.  workspace: the
// caller's device scratch of ws_bytes (may be NULL / 0: algorithms without workspace only).
extern "C" long long tm_conv1x1_workspace_bytes(void) { return kConv1x1MaxWorkspace; }

extern "C" int tm_conv1x1(int dtype, const void* x, const void* w, const void* bias, const void* residual,
                          void* y, long long rows, int cin, int cout, int relu, void* workspace, long long ws_bytes,
                          void* stream) {
  return conv1x1(Args{dtype, x, w, bias, residual, y, rows, cin, cout, relu, workspace, ws_bytes}, false,
                 (hipStream_t)stream);
}

extern "C" int tm_conv1x1_tune(int dtype, const void* x, const void* w, const void* bias, const void* residual,
                               void* y, long long rows, int cin, int cout, int relu, void* workspace,
                               long long ws_bytes, void* stream) {
  return conv1x1(Args{dtype, x, w, bias, residual, y, rows, cin, cout, relu, workspace, ws_bytes}, true,
                 (hipStream_t)stream);
}
