// Host side of the row queue (rowq.hpp) and the concurrency knobs of the row kernels,
// plus a diagnostic kernel that holds CUs the way a collective kernel does.
#include "common.hpp"
#include "rowq.hpp"

#include <atomic>
#include <cstdlib>
#include <mutex>

namespace gnnrec {
namespace {

constexpr int kMaxDevices = 64;
constexpr unsigned kRqSlots = 1024;  // launches that may be in flight on one device at once

std::atomic<int> g_reserve{0};
// the queue is the default schedule (gnnrec_set_concurrency(…, 0) selects the static
// grid-stride)
std::atomic<int> g_dynamic{1};
// a per-device ring of device scratch slots, zeroed once and left zeroed by each user's
// last block (self-cleaning); a slot is handed out only when its previous launch (on any
// stream) has completed — the event per slot — and never to a launch being captured
struct SlotRing {
  size_t slot_bytes;
  unsigned n_slots;
  std::mutex mu;
  std::atomic<char*> ring[kMaxDevices] = {};
  std::atomic<unsigned> next[kMaxDevices] = {};
  hipEvent_t* done[kMaxDevices] = {};
};
SlotRing g_rowq{(size_t)kRqSlotWords * sizeof(unsigned), kRqSlots};
SlotRing g_scan{(size_t)kScanSlotWords * sizeof(unsigned long long), kScanSlots};
std::atomic<long long> g_queued{0}, g_busy{0};  // row-queue launches given a slot / refused one
int g_cus[kMaxDevices] = {};

int current_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return dev >= 0 && dev < kMaxDevices ? dev : 0;
}

// `ticks` of the wall clock with the launch's dynamic LDS allocated: the residency of a
// collective kernel beside the row kernels (tools/probe_comm_overlap.py)
__global__ void hold_kernel(int64_t ticks, float* sink) {
  extern __shared__ float lds[];
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  const uint64_t t0 = wall_clock64();
  float acc = 0.f;
  while ((int64_t)(wall_clock64() - t0) < ticks) {
    acc += lds[(threadIdx.x + 1) % blockDim.x];
    __builtin_amdgcn_s_sleep(8);
  }
  if (acc < 0.f) sink[threadIdx.x] = acc;  // never taken: keeps the loop's loads
}

// nullptr: captured launch, allocation failure or busy slot (*busy set) — the caller then
// takes its slot-free path
char* ring_slot(SlotRing& r, hipStream_t stream, int* ticket, bool* busy) {
  *ticket = -1;
  *busy = false;
  // a launch captured into a hipGraph would replay with its slot baked in and no
  // completion check, so an eager launch could take the same slot while the replay runs
  // (two grids on one slot skip or repeat work): captured launches get no slot
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone)
    return nullptr;
  const int dev = current_device();
  char* ring = r.ring[dev].load(std::memory_order_acquire);
  if (ring == nullptr) {
    std::lock_guard<std::mutex> lk(r.mu);
    ring = r.ring[dev].load(std::memory_order_relaxed);
    if (ring == nullptr) {
      const size_t bytes = r.slot_bytes * r.n_slots;
      if (hipMalloc(&ring, bytes) != hipSuccess) return nullptr;
      hipEvent_t* ev = new hipEvent_t[r.n_slots]();
      bool ok = hipMemset(ring, 0, bytes) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
      for (unsigned i = 0; ok && i < r.n_slots; ++i)
        ok = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) == hipSuccess;
      if (!ok) {
        (void)hipFree(ring);
        return nullptr;
      }
      r.done[dev] = ev;
      r.ring[dev].store(ring, std::memory_order_release);
    }
  }
  const unsigned i = r.next[dev].fetch_add(1, std::memory_order_relaxed) % r.n_slots;
  // never recorded -> hipSuccess; still running -> hipErrorNotReady: no slot
  if (hipEventQuery(r.done[dev][i]) != hipSuccess) {
    *busy = true;
    return nullptr;
  }
  *ticket = (int)i;
  return ring + (size_t)i * r.slot_bytes;
}

void ring_launched(SlotRing& r, int ticket, hipStream_t stream) {
  if (ticket < 0) return;
  (void)hipEventRecord(r.done[current_device()][ticket], stream);
}

}  // namespace

int device_cus() {
  const int dev = current_device();
  if (g_cus[dev] == 0) {
    int n = 0;
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    g_cus[dev] = n > 0 ? n : 256;
  }
  return g_cus[dev];
}

int cu_reserve() { return g_reserve.load(std::memory_order_relaxed); }

unsigned* rowq_slot(hipStream_t stream, int* ticket) {
  *ticket = -1;
  if (!g_dynamic.load(std::memory_order_relaxed)) return nullptr;
  bool busy = false;
  char* q = ring_slot(g_rowq, stream, ticket, &busy);
  if (q) g_queued.fetch_add(1, std::memory_order_relaxed);
  else if (busy) g_busy.fetch_add(1, std::memory_order_relaxed);
  return reinterpret_cast<unsigned*>(q);  // nullptr: the static schedule
}

void rowq_launched(int ticket, hipStream_t stream) { ring_launched(g_rowq, ticket, stream); }

unsigned long long* scan_slot(hipStream_t stream, int* ticket) {
  bool busy = false;
  return reinterpret_cast<unsigned long long*>(ring_slot(g_scan, stream, ticket, &busy));
}

void scan_launched(int ticket, hipStream_t stream) { ring_launched(g_scan, ticket, stream); }


}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_set_concurrency(int reserve_cus, int dynamic) {
  GNNREC_REQUIRE(reserve_cus >= 0 && reserve_cus < 1024,
                 "gnnrec_set_concurrency: reserve_cus %d out of range", reserve_cus);
  g_reserve.store(reserve_cus);
  g_dynamic.store(dynamic ? 1 : 0);
  return GNNREC_OK;
}

extern "C" int gnnrec_get_concurrency(int* reserve_cus, int* dynamic) {
  GNNREC_REQUIRE(reserve_cus && dynamic, "gnnrec_get_concurrency: null pointer");
  *reserve_cus = g_reserve.load();
  *dynamic = g_dynamic.load();
  return GNNREC_OK;
}

extern "C" int gnnrec_rowq_stats(int64_t* queued, int64_t* busy) {
  GNNREC_REQUIRE(queued && busy, "gnnrec_rowq_stats: null pointer");
  *queued = g_queued.load();
  *busy = g_busy.load();
  return GNNREC_OK;
}

extern "C" int gnnrec_hold_cus(int blocks, int threads, int lds_bytes, int64_t usec,
                               float* sink, void* stream) {
  GNNREC_REQUIRE(blocks > 0 && blocks <= 4096 && threads >= 64 && threads <= 1024 &&
                     threads % 64 == 0 && lds_bytes >= threads * 4 && lds_bytes <= 64 * 1024 &&
                     usec >= 0 && usec <= 1000000 && sink,
                 "gnnrec_hold_cus: bad arguments");
  int khz = 0;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, current_device());
  const int64_t ticks = usec * (int64_t)(khz > 0 ? khz : 100000) / 1000;
  hipLaunchKernelGGL(hold_kernel, dim3(blocks), dim3(threads), (size_t)lds_bytes,
                     as_stream(stream), ticks, sink);
  return check_launch("gnnrec_hold_cus");
}
