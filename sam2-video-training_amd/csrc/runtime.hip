// Library metadata + in-library launch profiler.
//
// s2h_prof_enable(cap) pre-creates `cap` event pairs; while enabled every launch
// of a selected kind (s2h_prof_select mask: 1 attention forward, 2 attention
// backward, 4 GEMM; default 1) is bracketed by hipEventRecord on the stream it
// is launched on, together with its kind and shape.  bench.py reads the
// per-launch durations back with s2h_prof_read to price the dominant kernel
// against the bf16 MFMA roofline (no host sync inside the timed region).
#include "common.h"
#include <vector>
#include <mutex>

extern "C" int s2h_version() { return 1; }

namespace {
const uint64_t* g_rng_off = nullptr;
}
extern "C" int s2h_rng_bind(const void* dev_u64) {
  g_rng_off = (const uint64_t*)dev_u64;
  return 0;
}
const uint64_t* s2h_rng_offset_ptr() { return g_rng_off; }

namespace {
struct ProfRec { hipEvent_t a, b; int64_t meta[6]; int64_t tag; };
std::mutex g_mu;
std::vector<ProfRec> g_pool;
int g_used = 0;
bool g_on = false;
int g_mask = 1;
thread_local int t_slot = -1;  // the record the calling thread's current launch belongs to
}  // namespace

extern "C" int s2h_prof_enable(int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& r : g_pool) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  g_pool.clear();
  g_used = 0;
  g_on = cap > 0;
  for (int i = 0; i < cap; ++i) {
    ProfRec r;
    if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) return (int)hipErrorOutOfMemory;
    g_pool.push_back(r);
  }
  return 0;
}
extern "C" int s2h_prof_reset() { std::lock_guard<std::mutex> lk(g_mu); g_used = 0; return 0; }
extern "C" int s2h_prof_count() { std::lock_guard<std::mutex> lk(g_mu); return g_used; }

// internal: returns slot index or -1
extern "C" int s2h_prof_select(int mask) { std::lock_guard<std::mutex> lk(g_mu); g_mask = mask; return 0; }

// Launches on a capturing stream are not profiled: an event recorded there is only an
// intra-graph dependency, and hipEventRecordExternal is rejected in capture on ROCm 7.2.
static bool capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
static void record(hipEvent_t ev, hipStream_t st) { (void)hipEventRecord(ev, st); }

int s2h_prof_begin(hipStream_t st, int kind, int64_t m0, int64_t m1, int64_t m2, int64_t m3, int64_t m4) {
  if (!g_on || !(g_mask & kind) || capturing(st)) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_used >= (int)g_pool.size()) return -1;
  int i = g_used++;
  int64_t* m = g_pool[i].meta;
  m[0] = kind; m[1] = m0; m[2] = m1; m[3] = m2; m[4] = m3; m[5] = m4;
  g_pool[i].tag = 0;
  t_slot = i;
  record(g_pool[i].a, st);
  return i;
}
// the kernel the current record launches (called by the launchers once the tiling is chosen)
void s2h_prof_tag(int64_t tag) {
  if (t_slot >= 0) g_pool[t_slot].tag = tag;
}
void s2h_prof_end(int slot, hipStream_t st) {
  if (slot < 0) return;
  t_slot = -1;
  record(g_pool[slot].b, st);
}

extern "C" int s2h_prof_read_tags(int max, int64_t* tags) {
  std::lock_guard<std::mutex> lk(g_mu);
  int n = g_used < max ? g_used : max;
  for (int i = 0; i < n; ++i) tags[i] = g_pool[i].tag;
  return n;
}

// ms[i] = duration of record i; meta[6*i..] = (kind, shape[5]). Synchronises on the events.
extern "C" int s2h_prof_read(int max, float* ms, int64_t* meta) {
  std::lock_guard<std::mutex> lk(g_mu);
  int n = g_used < max ? g_used : max;
  for (int i = 0; i < n; ++i) {
    (void)hipEventSynchronize(g_pool[i].b);
    float t = 0.f;
    (void)hipEventElapsedTime(&t, g_pool[i].a, g_pool[i].b);
    ms[i] = t;
    for (int k = 0; k < 6; ++k) meta[6 * i + k] = g_pool[i].meta[k];
  }
  return n;
}

// Trace marker: a one-lane no-op kernel whose dispatch brackets a region in a rocprofv3 kernel
// trace (bench.py launches it right before and right after its timed steps; tools/step_profile.py
// keeps the kernels between the two).  rocprofv3 --selected-regions (ROCTx pause / resume) crashed
// at start-up on the ROCm 7.2 box, so the region is delimited in the trace itself.
__global__ void s2h_trace_marker_kernel(int tag) {
  if (tag == INT32_MIN) asm volatile("s_nop 0");  // never true: keeps the kernel non-empty
}
// With the profiler on and kind 8 selected the marker is a profiler record too: bench.py times
// bracketed empty launches to calibrate the per-record event overhead.
extern "C" int s2h_trace_marker(int tag, hipStream_t st) {
  const int slot = s2h_prof_begin(st, 8, tag, 0, 0, 0, 0);
  hipLaunchKernelGGL(s2h_trace_marker_kernel, dim3(1), dim3(64), 0, st, tag);
  s2h_prof_end(slot, st);
  return (int)hipGetLastError();
}
