// Deferred fixed-order gradient sums (round 5).
//
// The step's parameter gradients that come from a column reduction -- LayerNorm gamma / beta
// (norm.hip ln_bwd), the bias gradients of the short-reduction GEMMs and broadcast adds (s2h_colsum),
// the padded Hiera windows' qkv bias rows (s2h_window_pad_colsum) -- are computed in two passes: the
// first writes per-block partial rows, the second adds them in a fixed order into the gradient arena.
// The second pass is a ~5 us launch of a few KB of work, and a training step issued ~100 of them
// (profiles/r05_v13_kernel_stats.csv: ln_wgrad_finalize 71 + det_colsum ~30 per step).  Nothing in the
// backward reads a parameter gradient, so inside a deferral scope (s2h_grad_defer) the first pass writes
// its partials into a bump arena and the second pass is recorded; s2h_grad_defer_flush then adds every
// recorded reduction in a few launches (64 records per launch; a record whose destination overlaps an
// earlier record of the batch starts a new launch, so additions into one gradient keep their order).
// Only destinations inside the registered sink range (the gradient arena) are deferred; everything else
// keeps the immediate second pass.  The sum order inside a record is fixed by the record's shape:
// the result is deterministic (not bit-identical to the immediate pass, whose slice layout differs).
#include <vector>

#include "common.h"

namespace {

constexpr int kDeferMax = 64;  // records per flush launch (kernarg: 8 + 64 * 40 B)

struct DeferRec {
  const float* part;  // [nb][n0 + n1]
  float* out0;        // columns [0, n0)
  float* out1;        // columns [n0, n0 + n1) (nullptr when n1 == 0)
  int nb, n0, n1, blk0;  // blk0: first workgroup of this record in its launch
};
struct DeferBatch {
  int n, nblk;
  DeferRec r[kDeferMax];
};

// out[c] += sum_b part[b][c]: one workgroup per 64 columns of a record, 1024 threads = 64 columns x 16
// slices; slice s adds rows s, s + 16, ... in four independent chains (rows s + 64 j + 16 q, chain q),
// the chains are added in a fixed order, the 16 slice sums in a fixed LDS tree.
__global__ __launch_bounds__(1024) void grad_defer_flush_kernel(DeferBatch) {
  const DeferBatch* b = (const DeferBatch*)__builtin_amdgcn_kernarg_segment_ptr();
  int i = 0;
  while (i + 1 < b->n && b->r[i + 1].blk0 <= (int)blockIdx.x) ++i;
  const DeferRec& r = b->r[i];
  const int n = r.n0 + r.n1;
  const int col = ((int)blockIdx.x - r.blk0) * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;
  __shared__ float sh[16][64];
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
  if (col < n) {
    const float* p = r.part + col;
    int row = sl;
    for (; row + 48 < r.nb; row += 64) {
      c0 += p[(int64_t)row * n];
      c1 += p[(int64_t)(row + 16) * n];
      c2 += p[(int64_t)(row + 32) * n];
      c3 += p[(int64_t)(row + 48) * n];
    }
    if (row < r.nb) c0 += p[(int64_t)row * n];
    if (row + 16 < r.nb) c1 += p[(int64_t)(row + 16) * n];
    if (row + 32 < r.nb) c2 += p[(int64_t)(row + 32) * n];
  }
  sh[sl][threadIdx.x & 63] = (c0 + c1) + (c2 + c3);
  __syncthreads();
#pragma unroll
  for (int h = 8; h >= 1; h >>= 1) {
    if (sl < h) sh[sl][threadIdx.x & 63] += sh[sl + h][threadIdx.x & 63];
    __syncthreads();
  }
  if (sl == 0 && col < n) {
    float* o = col < r.n0 ? r.out0 + col : r.out1 + (col - r.n0);
    *o += sh[0][threadIdx.x & 63];
  }
}

struct DeferState {
  char* ws = nullptr;
  int64_t ws_bytes = 0, used = 0;
  uintptr_t sink_lo = 0, sink_hi = 0;
  std::vector<DeferRec> recs;
  hipStream_t st = nullptr;  // the stream of the scope's first record: every deferred record and flush runs on it
  bool have_st = false;
};
DeferState g_def;

bool in_sink(const float* p, int n) {
  const uintptr_t a = (uintptr_t)p;
  return p != nullptr && a >= g_def.sink_lo && a + (uintptr_t)n * sizeof(float) <= g_def.sink_hi;
}

bool overlaps(const DeferRec& a, const DeferRec& b) {
  auto ov = [](const float* p, int n, const float* q, int m) {
    return p && q && n > 0 && m > 0 && p < q + m && q < p + n;
  };
  return ov(a.out0, a.n0, b.out0, b.n0) || ov(a.out0, a.n0, b.out1, b.n1) || ov(a.out1, a.n1, b.out0, b.n0) ||
         ov(a.out1, a.n1, b.out1, b.n1);
}

int flush(hipStream_t st) {
  size_t k = 0;
  while (k < g_def.recs.size()) {
    DeferBatch batch;
    batch.n = 0;
    batch.nblk = 0;
    while (k < g_def.recs.size() && batch.n < kDeferMax) {
      DeferRec r = g_def.recs[k];
      bool clash = false;
      for (int j = 0; j < batch.n && !clash; ++j) clash = overlaps(batch.r[j], r);
      if (clash) break;
      r.blk0 = batch.nblk;
      batch.nblk += (r.n0 + r.n1 + 63) / 64;
      batch.r[batch.n++] = r;
      ++k;
    }
    hipLaunchKernelGGL(grad_defer_flush_kernel, dim3(batch.nblk), dim3(1024), 0, st, batch);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  g_def.recs.clear();
  g_def.used = 0;
  g_def.have_st = false;
  return 0;
}

}  // namespace

float* s2h_defer_sink(int nb, int n0, float* out0, int n1, float* out1, hipStream_t st) {
  if (g_def.ws == nullptr || nb <= 0 || n0 <= 0 || !in_sink(out0, n0) || (n1 > 0 && !in_sink(out1, n1)))
    return nullptr;
  // one stream per scope: a record from another stream (the opt-in weight-gradient side stream) keeps its
  // immediate second pass -- a mid-scope flush on one stream could read partials the other has not written
  // yet, and reuse workspace regions the other still reads
  if (g_def.have_st && st != g_def.st) return nullptr;
  const int64_t bytes = ((int64_t)nb * (n0 + n1) * (int64_t)sizeof(float) + 255) & ~(int64_t)255;
  if (bytes > g_def.ws_bytes) return nullptr;
  if (g_def.used + bytes > g_def.ws_bytes && flush(st) != 0) return nullptr;
  g_def.st = st;
  g_def.have_st = true;
  float* part = (float*)(g_def.ws + g_def.used);
  g_def.used += bytes;
  g_def.recs.push_back(DeferRec{part, out0, n1 > 0 ? out1 : nullptr, nb, n0, n1 > 0 ? n1 : 0, 0});
  return part;
}

// ws == nullptr ends the scope (every record must have been flushed: hipErrorNotReady otherwise).
extern "C" int s2h_grad_defer(void* ws, int64_t ws_bytes, void* sink, int64_t sink_bytes) {
  if (ws == nullptr) {
    if (!g_def.recs.empty()) return (int)hipErrorNotReady;
    g_def = DeferState{};
    return 0;
  }
  if (!g_def.recs.empty() || ws_bytes <= 0 || sink == nullptr || sink_bytes <= 0 || ((uintptr_t)ws & 255))
    return (int)hipErrorInvalidValue;
  g_def.ws = (char*)ws;
  g_def.ws_bytes = ws_bytes;
  g_def.used = 0;
  g_def.sink_lo = (uintptr_t)sink;
  g_def.sink_hi = (uintptr_t)sink + (uintptr_t)sink_bytes;
  return 0;
}

extern "C" int s2h_grad_defer_flush(hipStream_t st) {
  if (!g_def.recs.empty() && st != g_def.st) return (int)hipErrorInvalidResourceHandle;  // not the records' stream
  return flush(st);
}

// end the scope whatever is pending (records not flushed are dropped): the caller's cleanup after a failed
// flush, so later scopes can register
extern "C" int s2h_grad_defer_reset() {
  g_def = DeferState{};
  return 0;
}

extern "C" int s2h_grad_defer_pending() { return (int)g_def.recs.size(); }
