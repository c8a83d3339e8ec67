// C-ABI implementation (include/sks.h): contexts, sketch build orchestration,
// intersection launches and the host-side helpers of the reference API.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "sks.h"
#include "sks_api_internal.hpp"
#include "sks_hash.hpp"
#include "sks_ani.hpp"
#include "sks_internal.hpp"

namespace sks {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

namespace {
struct PinnedStage {
  void* p = nullptr;
  size_t bytes = 0;
};

// Host -> device copies of small metadata go through a pinned ring and do not
// wait: the bytes are copied into the ring at once (the caller's buffer may go
// away), the DMA is queued on `s`, and an event marks when that part of the
// ring may be rewritten.  A build used to synchronise its stream after every
// metadata upload (a dozen round trips for one 5 Mb genome).
struct RingUse {
  size_t off, len;
  int device;
  hipEvent_t ev;
};
struct PinnedRing {
  char* p = nullptr;
  size_t bytes = 0, head = 0;
  std::vector<RingUse> pending;
  std::vector<std::pair<int, hipEvent_t>> spare;  // (device, event) ready for reuse
};

// A thread's pinned staging (the d2h stage and the h2d ring).  Threads borrow
// one from a process-wide pool on first use and give it back when they exit,
// so the pinned memory is bounded by the largest number of threads staging at
// once, not by how many threads a long-running caller has started (the
// facade's parallel_* entry points start fresh threads on every call).  Pool
// entries are never freed: nothing touches HIP at thread or process exit
// (thread_local destructors of the main thread run before static ones, and
// could otherwise run after the HIP runtime is gone).
struct PinnedSlots {
  PinnedStage stage;
  PinnedRing ring;
};
std::mutex g_slots_mu;
std::vector<PinnedSlots*>* g_slots_pool = new std::vector<PinnedSlots*>();  // never freed

struct SlotsHandle {
  PinnedSlots* s = nullptr;
  PinnedSlots& get() {
    if (!s) {
      std::lock_guard<std::mutex> lk(g_slots_mu);
      if (!g_slots_pool->empty()) {
        s = g_slots_pool->back();
        g_slots_pool->pop_back();
      } else {
        s = new PinnedSlots();
      }
    }
    return *s;
  }
  ~SlotsHandle() {
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_slots_mu);
    g_slots_pool->push_back(s);  // pending ring copies stay tracked by their events
  }
};
thread_local SlotsHandle t_slots;

hipError_t stage_reserve(PinnedStage& st, size_t bytes) {
  if (bytes <= st.bytes) return hipSuccess;
  if (st.p) (void)hipHostFree(st.p);
  st.p = nullptr;
  st.bytes = 0;
  size_t nb = std::max<size_t>(bytes, size_t(1) << 16);
  nb = (nb + 4095) & ~size_t(4095);
  hipError_t e = hipHostMalloc(&st.p, nb, hipHostMallocDefault);
  if (e == hipSuccess) st.bytes = nb;
  return e;
}

void ring_retire(PinnedRing& R, size_t i) {
  R.spare.emplace_back(R.pending[i].device, R.pending[i].ev);
  R.pending.erase(R.pending.begin() + (std::ptrdiff_t)i);
}
}  // namespace

size_t pinned_pool_size() {
  std::lock_guard<std::mutex> lk(g_slots_mu);
  return g_slots_pool->size();
}

hipError_t pinned_d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  PinnedStage& st = t_slots.get().stage;
  hipError_t e;
  if ((e = stage_reserve(st, bytes)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(st.p, src, bytes, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  std::memcpy(dst, st.p, bytes);
  return hipSuccess;
}

hipError_t pinned_h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  PinnedRing& R = t_slots.get().ring;
  hipError_t e;
  int dev = 0;
  if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
  const size_t need = (bytes + 255) & ~size_t(255);
  // completed copies free their part of the ring
  for (size_t i = 0; i < R.pending.size();) {
    if (hipEventQuery(R.pending[i].ev) == hipSuccess) {
      ring_retire(R, i);
    } else {
      (void)hipGetLastError();  // hipErrorNotReady is not an error here
      ++i;
    }
  }
  if (need > R.bytes) {  // grow: drain, then reallocate
    for (const RingUse& u : R.pending)
      if ((e = hipEventSynchronize(u.ev)) != hipSuccess) return e;
    while (!R.pending.empty()) ring_retire(R, R.pending.size() - 1);
    if (R.p) (void)hipHostFree(R.p);
    R.p = nullptr;
    R.bytes = R.head = 0;
    const size_t nb = std::max<size_t>(4 * need, size_t(1) << 20);
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&R.p), nb, hipHostMallocDefault)) != hipSuccess)
      return e;
    R.bytes = nb;
  }
  if (R.head + need > R.bytes) R.head = 0;
  const size_t off = R.head;
  for (size_t i = 0; i < R.pending.size();) {  // copies still reading [off, off + need)
    const RingUse& u = R.pending[i];
    if (u.off < off + need && off < u.off + u.len) {
      if ((e = hipEventSynchronize(u.ev)) != hipSuccess) return e;
      ring_retire(R, i);
    } else {
      ++i;
    }
  }
  std::memcpy(R.p + off, src, bytes);
  if ((e = hipMemcpyAsync(dst, R.p + off, bytes, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
  hipEvent_t ev = nullptr;
  for (size_t i = 0; i < R.spare.size(); ++i)
    if (R.spare[i].first == dev) {
      ev = R.spare[i].second;
      R.spare.erase(R.spare.begin() + (std::ptrdiff_t)i);
      break;
    }
  if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
  if ((e = hipEventRecord(ev, s)) != hipSuccess) return e;
  R.pending.push_back({off, need, dev, ev});
  R.head = off + need;
  return hipSuccess;
}

}  // namespace sks

#define SKS_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return sks::fail(SKS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

#define SKS_TRY(expr)              \
  do {                             \
    int rc_ = (expr);              \
    if (rc_ != SKS_OK) return rc_; \
  } while (0)

struct sks_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr, ev_s0 = nullptr, ev_s1 = nullptr;
  hipEvent_t ev_i0 = nullptr, ev_i1 = nullptr;  // device FASTA ingress
  sks::Scratch ingress;             // per-line arrays of the device FASTA parser
  sks::Scratch tmp;                 // rocPRIM temporary storage
  sks::Scratch rec[3];              // scan records (key, val, hi)
  sks::Scratch buf[10];             // dense working columns
  sks::Scratch flag, pos;
  sks::Scratch meta;                // small per-segment device arrays
  sks::Scratch iwork;               // intersection bucket tables
  sks::Scratch tdone;               // fused ANI: workgroups finished per join tile
  sks::Scratch lay;                 // sks_all_pairs_ani: the join layout, its temp and packed counts
  const uint32_t* layout_stat = nullptr;  // the last join-layout build's 2 status words (in iwork)
  std::vector<uint64_t> meta_host;  // staging for `meta`
  sks_timings last{};
  int grid_override = 0;
  int intersect_algo = 0;  // sks::kIntersect*
  bool join_check = false;  // invariant-checking join / layout kernels (sks_ctx_set_join_check)
  uint32_t layout_blocks_hint = 0;  // sks_ctx_set_layout_blocks_hint (0: every block holds sketches)
  sks::Scratch root;                // sks_ctx_ani_table: ANI by shared-element count for one set size
  uint32_t root_size = 0;
  int root_k = 0;                   // 0: no table
};

struct sks_kmer_list {
  int device = 0;
  uint32_t n = 0;
  uint64_t total = 0;
  uint64_t* d_pos = nullptr;   // [total] window start byte of each k-mer, stream order
  uint64_t* d_bits = nullptr;  // [total][4] kmer_bits lo, hi, masked_bits lo, hi
  std::vector<uint64_t> counts;
};


namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Packs small host arrays into ctx->meta with one H2D copy.
class MetaArena {
 public:
  explicit MetaArena(sks_ctx* c) : c_(c) { c_->meta_host.clear(); }
  // reserve n words; returns the word offset
  size_t add(const std::vector<uint64_t>& v) {
    size_t o = c_->meta_host.size();
    c_->meta_host.insert(c_->meta_host.end(), v.begin(), v.end());
    c_->meta_host.push_back(0);  // keep every array non-empty
    return o;
  }
  size_t add_zero(size_t n) {
    size_t o = c_->meta_host.size();
    c_->meta_host.resize(o + n + 1, 0);
    return o;
  }
  int upload() {
    size_t bytes = c_->meta_host.size() * sizeof(uint64_t);
    SKS_HIP(c_->meta.reserve(bytes));
    SKS_HIP(sks::pinned_h2d(c_->meta.ptr, c_->meta_host.data(), bytes, c_->stream));
    return SKS_OK;
  }
  uint64_t* ptr(size_t off) const { return reinterpret_cast<uint64_t*>(c_->meta.ptr) + off; }

 private:
  sks_ctx* c_;
};

uint64_t* col(sks_ctx* c, int i) { return reinterpret_cast<uint64_t*>(c->buf[i].ptr); }

int reserve_cols(sks_ctx* c, std::initializer_list<int> ids, uint64_t words) {
  for (int i : ids) SKS_HIP(c->buf[i].reserve(std::max<uint64_t>(words, 1) * sizeof(uint64_t)));
  return SKS_OK;
}

int end_bit_of(uint64_t max_value) {
  int b = 64 - __builtin_clzll(max_value | 1);
  return b < 1 ? 1 : b;
}

std::vector<uint64_t> prefix(const std::vector<uint64_t>& v) {
  std::vector<uint64_t> o(v.size() + 1, 0);
  for (size_t i = 0; i < v.size(); ++i) o[i + 1] = o[i] + v[i];
  return o;
}

// One completed pass: final sketches of `segs` (global segment ids) in CSR.
struct PassOut {
  uint64_t* d = nullptr;          // elements (elem_words u64 each)
  size_t bytes = 0;               // allocation size of d
  std::vector<uint32_t> segs;
  std::vector<uint64_t> off;      // CSR in elements, size segs.size() + 1
};

// Device block cache for sketch arrays. hipFree of a sketch-sized array unmaps
// it (≈160 us for config 3's 24 MB set, measured with --hip-trace), more than
// the build's whole host-side post-processing; released arrays are parked here
// and handed to later builds instead. Blocks are plain hipMalloc memory.
struct CachedBlock {
  int device;
  void* p;
  size_t bytes;
  hipEvent_t ready;  // null, or the stream point after which the block is free
};
std::mutex g_cache_mu;
void trim_device_cache(int device);
std::vector<CachedBlock> g_cache;  // most recently released last
constexpr size_t kCacheMaxBlocks = 16;
constexpr size_t kCacheMaxBytes = size_t(4) << 30;

size_t cache_bytes_locked() {
  size_t t = 0;
  for (const auto& b : g_cache) t += b.bytes;
  return t;
}

int current_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

// A cached block of at least `bytes` (and at most 2x + 1 MB, so a small request
// does not pin a large block), or a fresh hipMalloc.
hipError_t dev_alloc(void** p, size_t bytes) {
  bytes = std::max<size_t>(bytes, 8);
  const int dev = current_device();
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    size_t best = g_cache.size();
    for (size_t i = 0; i < g_cache.size(); ++i) {
      CachedBlock& b = g_cache[i];
      if (b.device != dev || b.bytes < bytes || b.bytes > 2 * bytes + (size_t(1) << 20)) continue;
      if (b.ready) {  // stream-ordered release: reusable once its event has completed
        if (hipEventQuery(b.ready) != hipSuccess) {
          (void)hipGetLastError();  // hipErrorNotReady is not an error here
          continue;
        }
        (void)hipEventDestroy(b.ready);
        b.ready = nullptr;
      }
      if (best == g_cache.size() || b.bytes < g_cache[best].bytes) best = i;
    }
    if (best != g_cache.size()) {
      *p = g_cache[best].p;
      g_cache.erase(g_cache.begin() + best);
      return hipSuccess;
    }
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory) {  // give the cache back and retry once
    (void)hipGetLastError();
    trim_device_cache(dev);
    e = hipMalloc(p, bytes);
  }
  return e;
}

// Parks a block whose last use has completed (ready == null; the caller
// guarantees it, see sks_sketch_set_free) or completes at the event `ready`;
// evicts the oldest blocks beyond the cache limits (hipFree waits for them).
void dev_release(void* p, size_t bytes, hipEvent_t ready = nullptr) {
  if (!p) {
    if (ready) (void)hipEventDestroy(ready);
    return;
  }
  std::vector<CachedBlock> evict;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_cache.push_back({current_device(), p, std::max<size_t>(bytes, 8), ready});
    while (g_cache.size() > kCacheMaxBlocks ||
           (g_cache.size() > 1 && cache_bytes_locked() > kCacheMaxBytes)) {
      evict.push_back(g_cache.front());
      g_cache.erase(g_cache.begin());
    }
  }
  for (const CachedBlock& b : evict) {
    if (b.ready) (void)hipEventDestroy(b.ready);
    (void)hipFree(b.p);
  }
}

void trim_device_cache(int device) {
  std::vector<CachedBlock> drop;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (size_t i = 0; i < g_cache.size();) {
      if (g_cache[i].device == device) {
        drop.push_back(g_cache[i]);
        g_cache.erase(g_cache.begin() + i);
      } else {
        ++i;
      }
    }
  }
  for (const CachedBlock& b : drop) {
    if (b.ready) (void)hipEventDestroy(b.ready);
    (void)hipFree(b.p);
  }
}

// Returns a set's arrays to the block cache: at once (the device is idle for
// them), or ordered after the current end of `stream`.
void release_set_arrays(sks_sketch_set* set, hipStream_t stream, bool ordered) {
  uint64_t total = 0;
  for (uint32_t v : set->sizes) total += v;
  void* arrays[3] = {set->d_data, set->d_starts, set->d_sizes};
  const size_t bytes[3] = {std::max<uint64_t>(total * set->elem_words, 1) * 8,
                           (size_t)std::max<uint32_t>(set->n, 1) * 8,
                           (size_t)std::max<uint32_t>(set->n, 1) * 4};
  for (int i = 0; i < 3; ++i) {
    if (!arrays[i]) continue;
    hipEvent_t ev = nullptr;
    if (ordered) {
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
          hipEventRecord(ev, stream) != hipSuccess) {
        // no event: fall back to waiting for the stream, then release at once
        if (ev) (void)hipEventDestroy(ev);
        ev = nullptr;
        (void)hipGetLastError();
        (void)hipStreamSynchronize(stream);
      }
    }
    dev_release(arrays[i], bytes[i], ev);
  }
  set->d_data = nullptr;
  set->d_starts = nullptr;
  set->d_sizes = nullptr;
}

// Pass buffers are only used on the ctx stream, synchronised before this runs.
void free_passes(std::vector<PassOut>& passes) {
  for (auto& p : passes)
    if (p.d) dev_release(p.d, p.bytes);
  passes.clear();
}

}  // namespace

namespace sks {
hipError_t cache_alloc(void** p, size_t bytes) { return dev_alloc(p, bytes); }

void cache_release_after(void* p, size_t bytes, hipStream_t s) {
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(ev, s) != hipSuccess) {
    // no event: wait for the stream, then park the block as idle
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
    (void)hipGetLastError();
    (void)hipStreamSynchronize(s);
  }
  dev_release(p, bytes, ev);
}
}  // namespace sks

namespace {

int alloc_u64(uint64_t** p, uint64_t words, size_t* bytes_out = nullptr) {
  const size_t bytes = std::max<uint64_t>(words, 1) * sizeof(uint64_t);
  SKS_HIP(dev_alloc(reinterpret_cast<void**>(p), bytes));
  if (bytes_out) *bytes_out = bytes;
  return SKS_OK;
}

}  // namespace

namespace {

// The fused ANI store runs in k_join: the caller's matrix must be memory the
// device can write — device memory, managed memory, or pinned host memory
// mapped into the device (sks_host_alloc), whose device-side address is
// returned.  An ordinary malloc/numpy buffer is refused (SKS_E_ARG) instead of
// being handed to the kernel, where the store would fault (XNACK is off).
int device_view_of_ani(double* ani, double** d_ani, const char* who) {
  hipPointerAttribute_t at{};
  const hipError_t e = hipPointerGetAttributes(&at, ani);
  (void)hipGetLastError();  // an unknown pointer leaves an error behind
  if (e != hipSuccess || at.type == hipMemoryTypeUnregistered)
    return sks::fail(SKS_E_ARG, std::string(who) + ": the ANI matrix is neither device memory nor pinned "
                                "host memory mapped into the device (use sks_host_alloc)");
  if (at.type == hipMemoryTypeHost) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, ani, 0) != hipSuccess || !dp) {
      (void)hipGetLastError();
      return sks::fail(SKS_E_ARG, std::string(who) + ": the pinned host ANI matrix is not mapped into the "
                                  "device (use sks_host_alloc)");
    }
    *d_ani = static_cast<double*>(dp);
  } else {
    *d_ani = ani;
  }
  return SKS_OK;
}

}  // namespace

extern "C" {

int sks_abi_version(void) { return SKS_ABI_VERSION; }

const char* sks_last_error(void) { return sks::g_last_error.c_str(); }

// ---- host helpers -----------------------------------------------------------------------

// kmer_bitset.cpp:132-152 — std::shuffle(iota(w), std::mt19937(seed)); the
// first k shuffled indices j set mask bits 2j and 2j+1.  libstdc++ is used on
// purpose: the reference's masks are defined by its shuffle algorithm.
int sks_mask_generate(int window, int k, uint64_t seed, uint64_t mask[2]) {
  if (!mask) return sks::fail(SKS_E_ARG, "sks_mask_generate: null mask");
  if (window < 1 || window > 64 || k < 0 || k > window)
    return sks::fail(SKS_E_ARG, "sks_mask_generate: need 0 <= k <= window <= 64");
  std::vector<int> idx(window);
  std::iota(idx.begin(), idx.end(), 0);
  std::shuffle(idx.begin(), idx.end(), std::mt19937((std::mt19937::result_type)seed));
  mask[0] = mask[1] = 0;
  for (int i = 0; i < k; ++i) {
    int b = 2 * idx[i];
    mask[b >> 6] |= 3ull << (b & 63);
  }
  return SKS_OK;
}

// kmer_bitset.cpp:50-56 — 2l low bits set; l > 64 throws in the reference.
int sks_mask_contiguous(int length, uint64_t mask[2]) {
  if (!mask) return sks::fail(SKS_E_ARG, "sks_mask_contiguous: null mask");
  if (length > 64) return sks::fail(SKS_E_ARG, "Given k-mer length exceeds maximum k-mer length");
  if (length < 0) return sks::fail(SKS_E_ARG, "sks_mask_contiguous: negative length");
  int bits = 2 * length;
  mask[0] = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
  mask[1] = bits <= 64 ? 0 : (bits >= 128 ? ~0ull : ((1ull << (bits - 64)) - 1));
  return SKS_OK;
}

uint64_t sks_frac_min_hash(const uint64_t kmer[2], const uint64_t mask[2], int window,
                           int64_t nonce, int flavour) {
  return sks::hash_bitset128_rt(kmer[0], kmer[1], flavour) ^
         sks::fmh_const(mask[0], mask[1], window, nonce, flavour);
}

double sks_containment(int intersection, int set_size) {
  if (intersection == 0) return 0;
  return ((double)intersection) / ((double)set_size);
}

double sks_binomial_estimator(double containment, int kmer_num_ones) {
  if (containment <= 0) return 0;
  return std::pow(containment, ((double)1.0) / ((double)kmer_num_ones));
}

int sks_ani_from_counts(const int32_t* inter, const int32_t* size_first, uint64_t n,
                        int kmer_num_ones, double* cont, double* ani) {
  if (n && (!inter || !size_first)) return sks::fail(SKS_E_ARG, "sks_ani_from_counts: null input");
  // element-wise and order-free: large batches (an all-vs-all matrix) are split
  // over host threads; every element is the same scalar double arithmetic
  auto run = [=](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      double c = sks_containment(inter[i], size_first[i]);
      if (cont) cont[i] = c;
      if (ani) ani[i] = sks_binomial_estimator(c, kmer_num_ones);
    }
  };
  const uint64_t kPer = 8192;
  unsigned T = std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  T = (unsigned)std::min<uint64_t>(T, (n + kPer - 1) / kPer);
  if (T <= 1) {
    run(0, n);
    return SKS_OK;
  }
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < T; ++t) pool.emplace_back(run, n * t / T, n * (t + 1) / T);
  run(0, n / T);
  for (auto& th : pool) th.join();
  return SKS_OK;
}

// ---- contexts -----------------------------------------------------------------------------

int sks_ctx_create(int device, void* stream, sks_ctx** out) {
  if (!out) return sks::fail(SKS_E_ARG, "sks_ctx_create: null out");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return sks::fail(SKS_E_HIP, std::string("sks_ctx_create: no HIP device available (the engine has "
                                            "no CPU path): hipGetDeviceCount -> ") +
                                    hipGetErrorString(e) + ", " + std::to_string(n) + " devices");
  if (device < 0 || device >= n) return sks::fail(SKS_E_ARG, "sks_ctx_create: bad device index");
  DeviceGuard g(device);
  sks_ctx* c = new (std::nothrow) sks_ctx();
  if (!c) return sks::fail(SKS_E_NOMEM, "sks_ctx_create: out of memory");
  c->device = device;
  c->stream = reinterpret_cast<hipStream_t>(stream);
  // every scratch buffer is used on the context's stream only
  for (sks::Scratch* sc : {&c->ingress, &c->tmp, &c->rec[0], &c->rec[1], &c->rec[2], &c->flag,
                           &c->pos, &c->meta, &c->iwork, &c->tdone, &c->lay, &c->root})
    sc->owner = &c->stream;
  for (auto& b : c->buf) b.owner = &c->stream;
  if (hipEventCreate(&c->ev_begin) != hipSuccess || hipEventCreate(&c->ev_end) != hipSuccess ||
      hipEventCreate(&c->ev_s0) != hipSuccess || hipEventCreate(&c->ev_s1) != hipSuccess ||
      hipEventCreate(&c->ev_i0) != hipSuccess || hipEventCreate(&c->ev_i1) != hipSuccess) {
    delete c;
    return sks::fail(SKS_E_HIP, "sks_ctx_create: hipEventCreate failed");
  }
  // every code object of the library on this device, before the first build
#define SKS_CALL_HOOK(tu) \
  if (e == hipSuccess) e = sks::code_object_hook_##tu(c->stream);
  e = hipSuccess;
  SKS_TU_LIST(SKS_CALL_HOOK)
#undef SKS_CALL_HOOK
  if (e != hipSuccess) {
    delete c;
    return sks::fail(SKS_E_HIP, std::string("sks_ctx_create: code object load: ") + hipGetErrorString(e));
  }
  *out = c;
  return SKS_OK;
}

int sks_ctx_destroy(sks_ctx* c) {
  if (!c) return SKS_OK;
  DeviceGuard g(c->device);
  (void)hipStreamSynchronize(c->stream);
  c->tmp.release();
  for (auto& r : c->rec) r.release();
  for (auto& b : c->buf) b.release();
  c->flag.release();
  c->pos.release();
  c->meta.release();
  c->iwork.release();
  c->tdone.release();
  c->lay.release();
  c->root.release();
  c->ingress.release();
  trim_device_cache(c->device);
  (void)hipEventDestroy(c->ev_begin);
  (void)hipEventDestroy(c->ev_end);
  (void)hipEventDestroy(c->ev_s0);
  (void)hipEventDestroy(c->ev_s1);
  if (c->ev_i0) (void)hipEventDestroy(c->ev_i0);
  if (c->ev_i1) (void)hipEventDestroy(c->ev_i1);
  delete c;
  return SKS_OK;
}

int sks_ctx_device(const sks_ctx* c) { return c ? c->device : -1; }

int sks_ctx_set_stream(sks_ctx* c, void* stream) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ctx_set_stream: null ctx");
  // scratch blocks are released in the order of the context's stream: let the
  // old stream's work finish before the order changes
  if (c->stream != reinterpret_cast<hipStream_t>(stream)) {
    DeviceGuard g(c->device);
    SKS_HIP(hipStreamSynchronize(c->stream));
  }
  c->stream = reinterpret_cast<hipStream_t>(stream);
  return SKS_OK;
}

int sks_ctx_synchronize(sks_ctx* c) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ctx_synchronize: null ctx");
  DeviceGuard g(c->device);
  SKS_HIP(hipStreamSynchronize(c->stream));
  return SKS_OK;
}

int sks_ctx_last_timings(const sks_ctx* c, sks_timings* out) {
  if (!c || !out) return sks::fail(SKS_E_ARG, "sks_ctx_last_timings: null argument");
  *out = c->last;
  return SKS_OK;
}

// Test/bench knob (not in sks.h): fixed scan grid size, 0 = occupancy-derived.
int sks_ctx_set_scan_grid(sks_ctx* c, int grid) {
  if (!c) return sks::fail(SKS_E_ARG, "null ctx");
  c->grid_override = grid;
  return SKS_OK;
}

int sks_ctx_set_intersect_kernel(sks_ctx* c, int kind) {
  if (!c) return sks::fail(SKS_E_ARG, "null ctx");
  if (kind < SKS_INTERSECT_AUTO || kind > SKS_INTERSECT_GLOBAL)
    return sks::fail(SKS_E_ARG, "sks_ctx_set_intersect_kernel: unknown kernel");
  c->intersect_algo = kind;
  return SKS_OK;
}

int sks_ctx_set_layout_blocks_hint(sks_ctx* c, uint32_t blocks) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ctx_set_layout_blocks_hint: null ctx");
  c->layout_blocks_hint = blocks;
  return SKS_OK;
}

int sks_ctx_ani_table(sks_ctx* c, uint32_t size, int kmer_num_ones) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ctx_ani_table: null ctx");
  if (kmer_num_ones <= 0) return sks::fail(SKS_E_ARG, "sks_ctx_ani_table: kmer_num_ones must be positive");
  if (size == 0 || size > SKS_ANI_TABLE_MAX) {
    c->root_k = 0;
    return SKS_OK;
  }
  if (c->root_k == kmer_num_ones && c->root_size == size) return SKS_OK;  // already built (stream order)
  DeviceGuard g(c->device);
  SKS_HIP(c->root.reserve(((size_t)size + 1) * sizeof(double)));
  SKS_HIP(sks::launch_ani_root(static_cast<double*>(c->root.ptr), size, kmer_num_ones, c->stream));
  c->root_size = size;
  c->root_k = kmer_num_ones;
  return SKS_OK;
}

int sks_ctx_set_join_check(sks_ctx* c, int on) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ctx_set_join_check: null ctx");
  c->join_check = on != 0;
  return SKS_OK;
}

int sks_ctx_join_check_violations(sks_ctx* c, uint64_t* violations) {
  if (!c || !violations) return sks::fail(SKS_E_ARG, "sks_ctx_join_check_violations: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(hipStreamSynchronize(c->stream));
  *violations = sks::join_check_take() + sks::layout_check_take();
  return SKS_OK;
}

}  // extern "C"

// ---- sketch build ---------------------------------------------------------------------------
namespace {

struct BuildState {
  sks_ctx* c;
  int w;
  bool wide;
  int ew;
  uint64_t mask_lo, mask_hi;
  sks_policy pol;
  uint64_t kconst;
  sks::DivTest dt;
};

// Post-process the segments `ok` (pass-local indices into the pass arrays) whose
// survivors sit in the record regions [out_off[i], out_off[i] + count[i]).
// Appends a PassOut; for bottom-s reports segments that need a larger threshold.
int post_process(BuildState& S, const std::vector<uint32_t>& seg_ids,
                 const std::vector<uint64_t>& out_off, const std::vector<uint64_t>& counts,
                 const std::vector<uint64_t>& thresh, const std::vector<uint32_t>& ok,
                 std::vector<PassOut>& passes, std::vector<uint32_t>& retry_local,
                 std::vector<uint64_t>& final_size_local) {
  sks_ctx* c = S.c;
  hipStream_t st = c->stream;
  const uint32_t k = (uint32_t)ok.size();
  if (k == 0) return SKS_OK;
  std::vector<uint64_t> src_off(k), cnt(k);
  uint64_t max_len = 0;
  for (uint32_t i = 0; i < k; ++i) {
    src_off[i] = out_off[ok[i]];
    cnt[i] = counts[ok[i]];
    max_len = std::max(max_len, cnt[i]);
  }
  std::vector<uint64_t> csr = prefix(cnt);
  const uint64_t T = csr[k];
  const bool bottom = S.pol.kind == SKS_BOTTOM_S;

  MetaArena arena(c);
  size_t o_src = arena.add(src_off), o_csr = arena.add(csr), o_uniq = arena.add_zero(k);
  // narrow bottom-s with every genome's candidates in one workgroup's registers:
  // sort, unique and select per genome in one kernel (post.hip k_bottom_fused).
  // A single genome goes the device-wide way instead: one workgroup sorting its
  // ~1.1 s candidates alone takes longer than the multi-workgroup radix sort
  // (config 2: 0.35 vs 0.30 ms per build; from two genomes on the fused kernel
  // wins, tools/ab_c2.sh)
  const bool fused = bottom && !S.wide && max_len <= sks::bottom_fused_capacity() &&
                     (k >= 2 || getenv("SKS_FUSED_SINGLE") != nullptr) &&
                     getenv("SKS_NO_FUSED_BOTTOM") == nullptr;
  std::vector<uint64_t> f_retry, f_pad(1, 0);
  size_t o_cnt = 0, o_retry = 0, o_pad = 0, o_res = 0;
  if (fused) {
    for (uint32_t i = 0; i < k; ++i) {
      f_retry.push_back(thresh[ok[i]] != ~0ull ? 1 : 0);
      f_pad.push_back(f_pad.back() + std::min<uint64_t>(S.pol.param, cnt[i]));
    }
    o_cnt = arena.add(cnt);
    o_retry = arena.add(f_retry);
    o_pad = arena.add(f_pad);
    o_res = arena.add_zero(k);
  }
  SKS_TRY(arena.upload());
  uint64_t* d_src = arena.ptr(o_src);
  uint64_t* d_csr = arena.ptr(o_csr);
  uint64_t* d_uniq = arena.ptr(o_uniq);

  if (fused) {
    SKS_TRY(reserve_cols(c, {5}, f_pad[k] + 1));
    const sks::BitRuns runs = sks::bit_runs(S.mask_lo);
    const int kb = std::max(1, __builtin_popcountll(S.mask_lo));
    SKS_HIP(sks::launch_bottom_fused(reinterpret_cast<uint64_t*>(c->rec[0].ptr), d_src,
                                     arena.ptr(o_cnt), arena.ptr(o_retry), arena.ptr(o_pad), k,
                                     max_len, S.pol.param, kb, runs, S.kconst, S.pol.flavour, col(c, 5),
                                     arena.ptr(o_res), st));
    std::vector<uint64_t> res(k);
    SKS_HIP(sks::pinned_d2h(res.data(), arena.ptr(o_res), k * sizeof(uint64_t), st));
    PassOut po;
    std::vector<uint64_t> limit(k, 0), keep_off(1, 0);
    uint64_t max_lim = 0;
    for (uint32_t i = 0; i < k; ++i) {
      if (res[i] == ~0ull) {
        retry_local.push_back(ok[i]);  // too few distinct candidates under the threshold
        continue;
      }
      limit[i] = res[i];
      max_lim = std::max(max_lim, res[i]);
      final_size_local[ok[i]] = res[i];
      po.segs.push_back(seg_ids[ok[i]]);
      keep_off.push_back(keep_off.back() + res[i]);
    }
    std::vector<uint64_t> dense = prefix(limit);
    MetaArena arena2(c);  // uploads are stream-ordered: safe to rewrite the arena
    const size_t o_psrc = arena2.add(f_pad), o_pdst = arena2.add(dense);
    SKS_TRY(arena2.upload());
    SKS_TRY(alloc_u64(&po.d, dense[k], &po.bytes));
    SKS_HIP(sks::compact_regions(col(c, 5), po.d, arena2.ptr(o_psrc), arena2.ptr(o_pdst), k,
                                 max_lim, st));
    po.off = keep_off;
    // no stream sync: the pass's outputs are consumed in stream order
    passes.push_back(po);
    return SKS_OK;
  }

  SKS_TRY(reserve_cols(c, {0, 1, 2, 3, 4, 5, 6, 7, 8, 9}, T + 1));
  SKS_HIP(c->flag.reserve((T + 1) * sizeof(uint32_t)));
  SKS_HIP(c->pos.reserve((T + 1) * sizeof(uint64_t)));
  uint32_t* d_flag = reinterpret_cast<uint32_t*>(c->flag.ptr);
  uint64_t* d_pos = reinterpret_cast<uint64_t*>(c->pos.ptr);
  const uint64_t* rk = reinterpret_cast<uint64_t*>(c->rec[0].ptr);
  const uint64_t* rv = reinterpret_cast<uint64_t*>(c->rec[1].ptr);
  const uint64_t* rh = reinterpret_cast<uint64_t*>(c->rec[2].ptr);

  // dense columns; narrow keys are packed to their mask bits for the sorts
  // (sks::BitRuns) and expanded again when the unique elements are scattered
  const sks::BitRuns runs = S.wide ? sks::BitRuns{} : sks::bit_runs(S.mask_lo);
  const int key_bits = S.wide ? 64 : std::max(1, __builtin_popcountll(S.mask_lo));
  const int mask_lo_bits = end_bit_of(S.mask_lo);
  const int mask_hi_bits = end_bit_of(S.mask_hi);
  // FracMinHash over several genomes: the segment index rides above the key (or,
  // 128-bit, above the high word) and every sort below is ONE device-wide radix
  // sort over all segments (compact_regions); a segmented sort gives each genome
  // one workgroup (reference sweep, 64 x 5 Mb at c = 200: 0.50 ms per narrow
  // sort, 2 x 0.68 ms per 128-bit one)
  const int tag_bits = sks::seg_tag_bits(k);
  const int tag_at = S.wide ? mask_hi_bits : key_bits;
  const bool tagged = !bottom && k >= 2 && tag_at + tag_bits <= 64 && getenv("SKS_SEGMENTED_SORT") == nullptr;
  const std::vector<uint64_t> one_seg{0, T};
  const std::vector<uint64_t>& sort_off = tagged ? one_seg : csr;
  const uint64_t* d_sort_off = tagged ? nullptr : d_csr;
  const uint64_t keep = tag_at >= 64 ? ~0ull : (1ull << tag_at) - 1;  // the key bits below the tag
  SKS_HIP(sks::compact_regions(rk, col(c, 0), d_src, d_csr, k, max_len, st, &runs,
                               tagged && !S.wide ? key_bits : -1));
  // narrow bottom-s records carry the k-mer as key (its fmh is recomputed here)
  const bool has_val = S.wide || (bottom && S.wide);
  if (has_val)
    SKS_HIP(sks::compact_regions(rv, col(c, 1), d_src, d_csr, k, max_len, st, nullptr, tagged ? mask_hi_bits : -1));
  if (bottom && S.wide) SKS_HIP(sks::compact_regions(rh, col(c, 2), d_src, d_csr, k, max_len, st));

  uint64_t max_thr = 0;
  for (uint32_t i = 0; i < k; ++i) max_thr = std::max(max_thr, thresh[ok[i]]);

  PassOut po;
  for (uint32_t i = 0; i < k; ++i) po.segs.push_back(seg_ids[ok[i]]);
  std::vector<uint64_t> uniq(k);

  if (!bottom) {
    const uint64_t* K;   // sorted unique columns source
    const uint64_t* K2 = nullptr;
    if (!S.wide && (tagged || k < 2 || getenv("SKS_SEGMENTED_SORT"))) {
      SKS_HIP(sks::seg_sort_keys(col(c, 0), col(c, 3), T, sort_off, d_sort_off,
                                 key_bits + (tagged ? tag_bits : 0), c->tmp, st));
      K = col(c, 3);
    } else if (!S.wide) {
      // keys too wide for a tag above them (2k + tag bits > 64): two stable
      // device-wide passes, by key with the segment as value, then by segment
      SKS_HIP(sks::launch_seg_ids(col(c, 1), d_csr, k, max_len, st));
      SKS_HIP(sks::seg_sort_pairs(col(c, 0), col(c, 3), col(c, 1), col(c, 4), T, one_seg, nullptr, key_bits,
                                  c->tmp, st));
      SKS_HIP(sks::seg_sort_pairs(col(c, 4), col(c, 5), col(c, 3), col(c, 6), T, one_seg, nullptr,
                                  std::max(1, tag_bits), c->tmp, st));
      K = col(c, 6);
    } else {
      // (lo, hi) -> sort by lo, then stable by hi  => ascending 128-bit order
      SKS_HIP(sks::seg_sort_pairs(col(c, 0), col(c, 3), col(c, 1), col(c, 4), T, sort_off, d_sort_off,
                                  mask_lo_bits, c->tmp, st));
      SKS_HIP(sks::seg_sort_pairs(col(c, 4), col(c, 5), col(c, 3), col(c, 6), T, sort_off, d_sort_off,
                                  mask_hi_bits + (tagged ? tag_bits : 0), c->tmp, st));
      K = col(c, 5);   // hi (tagged)
      K2 = col(c, 6);  // lo
    }
    SKS_HIP(sks::seg_unique_scan(K, K2, T, max_len, d_csr, k, d_flag, d_pos, d_uniq, c->tmp, st));
    SKS_HIP(sks::pinned_d2h(uniq.data(), d_uniq, k * sizeof(uint64_t), st));
    po.off = prefix(uniq);
    const uint64_t U = po.off[k];
    SKS_TRY(alloc_u64(&po.d, U * S.ew, &po.bytes));
    if (!S.wide) {
      SKS_HIP(sks::seg_unique_scatter(K, nullptr, T, max_len, d_csr, k, d_flag, d_pos, nullptr, nullptr,
                                      po.d, nullptr, st, &runs, keep));
    } else {
      SKS_HIP(sks::seg_unique_scatter(K2, K, T, max_len, d_csr, k, d_flag, d_pos, nullptr, nullptr,
                                      col(c, 7), col(c, 8), st, nullptr, ~0ull, keep));
      SKS_HIP(sks::launch_interleave(col(c, 7), col(c, 8), U, po.d, st));
    }
    for (uint32_t i = 0; i < k; ++i) final_size_local[ok[i]] = uniq[i];
    passes.push_back(po);
    return SKS_OK;
  }

  // bottom-s
  const uint64_t s = S.pol.param;
  if (!S.wide) {
    // sort the candidate k-mers, unique them, then select the s with the smallest
    // (fmh, k-mer) per genome in LDS (k_bottom_select, post.hip): one key-only
    // sort instead of a (fmh, k-mer) pair sort followed by a second sort
    SKS_HIP(sks::seg_sort_keys(col(c, 0), col(c, 3), T, csr, d_csr, key_bits, c->tmp, st));
    SKS_HIP(sks::seg_unique_scan(col(c, 3), nullptr, T, max_len, d_csr, k, d_flag, d_pos, d_uniq,
                                 c->tmp, st));
    SKS_HIP(sks::pinned_d2h(uniq.data(), d_uniq, k * sizeof(uint64_t), st));
    uint64_t max_keep_uniq = 0;
    for (uint32_t i = 0; i < k; ++i)
      if (uniq[i] >= s || thresh[ok[i]] == ~0ull) max_keep_uniq = std::max(max_keep_uniq, uniq[i]);
    if (max_keep_uniq <= sks::bottom_select_capacity()) {
      std::vector<uint64_t> limit(k, 0);
      std::vector<uint32_t> keep_segs;
      std::vector<uint64_t> keep_off(1, 0);
      for (uint32_t i = 0; i < k; ++i) {
        if (uniq[i] >= s || thresh[ok[i]] == ~0ull) {
          limit[i] = std::min<uint64_t>(s, uniq[i]);
          final_size_local[ok[i]] = limit[i];
          keep_segs.push_back(seg_ids[ok[i]]);
          keep_off.push_back(keep_off.back() + limit[i]);
        } else {
          retry_local.push_back(ok[i]);  // too few candidates under the threshold
        }
      }
      std::vector<uint64_t> dst = prefix(limit), uoff = prefix(uniq);
      const uint64_t U = dst[k];
      // every distinct candidate, contiguous per genome at uoff
      SKS_HIP(sks::seg_unique_scatter(col(c, 3), nullptr, T, max_len, d_csr, k, d_flag, d_pos,
                                      nullptr, nullptr, col(c, 5), nullptr, st, &runs));
      MetaArena arena2(c);  // uploads are stream-ordered: safe to rewrite the arena
      size_t o_uoff = arena2.add(uoff), o_lim = arena2.add(limit), o_dst = arena2.add(dst);
      SKS_TRY(arena2.upload());
      SKS_TRY(alloc_u64(&po.d, U, &po.bytes));
      po.segs = keep_segs;
      po.off = keep_off;
      SKS_HIP(sks::launch_bottom_select(col(c, 5), arena2.ptr(o_uoff), arena2.ptr(o_dst),
                                        arena2.ptr(o_lim), k, S.kconst, S.pol.flavour, po.d, st));
      // no stream sync: the pass's outputs are consumed in stream order
      passes.push_back(po);
      return SKS_OK;
    }
    // a genome with more distinct candidates than the LDS select holds: the
    // general path below, on (fmh, k-mer) pairs
    SKS_HIP(sks::launch_bits_expand(col(c, 0), T, runs, st));
    SKS_HIP(hipMemcpyAsync(col(c, 1), col(c, 0), T * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    SKS_HIP(sks::launch_fmh_narrow(col(c, 0), T, S.kconst, S.pol.flavour, st));
  }
  const uint64_t* LO;  // columns ordered by (fmh, C)
  const uint64_t* HI = nullptr;
  if (!S.wide) {
    SKS_HIP(sks::seg_sort_pairs(col(c, 0), col(c, 3), col(c, 1), col(c, 4), T, csr, d_csr,
                                end_bit_of(max_thr), c->tmp, st));
    LO = col(c, 4);
    SKS_HIP(sks::seg_unique_scan(col(c, 3), nullptr, T, max_len, d_csr, k, d_flag, d_pos, d_uniq,
                                 c->tmp, st));
  } else {
    // order (fmh, hi, lo) by an index permutation (LSD: lo, hi, fmh)
    uint64_t* idx = col(c, 9);
    SKS_HIP(sks::launch_iota(idx, T, st));
    SKS_HIP(sks::seg_sort_pairs(col(c, 1), col(c, 3), idx, col(c, 4), T, csr, d_csr, 64, c->tmp, st));
    SKS_HIP(sks::launch_gather(col(c, 2), col(c, 4), T, col(c, 5), st));
    SKS_HIP(sks::seg_sort_pairs(col(c, 5), col(c, 3), col(c, 4), col(c, 6), T, csr, d_csr,
                                mask_hi_bits, c->tmp, st));
    SKS_HIP(sks::launch_gather(col(c, 0), col(c, 6), T, col(c, 5), st));
    SKS_HIP(sks::seg_sort_pairs(col(c, 5), col(c, 3), col(c, 6), col(c, 4), T, csr, d_csr,
                                end_bit_of(max_thr), c->tmp, st));
    SKS_HIP(sks::launch_gather(col(c, 1), col(c, 4), T, col(c, 7), st));  // lo
    SKS_HIP(sks::launch_gather(col(c, 2), col(c, 4), T, col(c, 8), st));  // hi
    LO = col(c, 7);
    HI = col(c, 8);
    SKS_HIP(sks::seg_unique_scan(LO, HI, T, max_len, d_csr, k, d_flag, d_pos, d_uniq, c->tmp, st));
  }
  SKS_HIP(sks::pinned_d2h(uniq.data(), d_uniq, k * sizeof(uint64_t), st));
  std::vector<uint64_t> limit(k, 0);
  std::vector<uint32_t> keep_segs;
  std::vector<uint64_t> keep_off(1, 0);
  for (uint32_t i = 0; i < k; ++i) {
    const bool done = uniq[i] >= s || thresh[ok[i]] == ~0ull;
    if (done) {
      limit[i] = std::min<uint64_t>(s, uniq[i]);
      final_size_local[ok[i]] = limit[i];
      keep_segs.push_back(seg_ids[ok[i]]);
      keep_off.push_back(keep_off.back() + limit[i]);
    } else {
      retry_local.push_back(ok[i]);  // too few candidates under the threshold
    }
  }
  // not-done segments get limit 0, so this prefix is also keep_off's layout
  std::vector<uint64_t> dst = prefix(limit);
  const uint64_t U = dst[k];
  MetaArena arena2(c);  // uploads are stream-ordered: safe to rewrite the arena
  size_t o_csr2 = arena2.add(csr), o_lim = arena2.add(limit), o_dst = arena2.add(dst);
  SKS_TRY(arena2.upload());
  d_csr = arena2.ptr(o_csr2);
  uint64_t* d_lim = arena2.ptr(o_lim);
  uint64_t* d_dst = arena2.ptr(o_dst);
  SKS_TRY(alloc_u64(&po.d, U * S.ew, &po.bytes));
  po.segs = keep_segs;
  po.off = keep_off;
  if (!S.wide) {
    SKS_HIP(sks::seg_unique_scatter(LO, nullptr, T, max_len, d_csr, k, d_flag, d_pos, d_lim, d_dst,
                                    col(c, 5), nullptr, st));
    SKS_HIP(sks::seg_sort_keys(col(c, 5), po.d, U, dst, d_dst, mask_lo_bits, c->tmp, st));
  } else {
    SKS_HIP(sks::seg_unique_scatter(LO, HI, T, max_len, d_csr, k, d_flag, d_pos, d_lim, d_dst, col(c, 0),
                                    col(c, 1), st));
    SKS_HIP(sks::seg_sort_pairs(col(c, 0), col(c, 3), col(c, 1), col(c, 4), U, dst, d_dst, 64,
                                c->tmp, st));
    SKS_HIP(sks::seg_sort_pairs(col(c, 4), col(c, 5), col(c, 3), col(c, 6), U, dst, d_dst,
                                mask_hi_bits, c->tmp, st));
    SKS_HIP(sks::launch_interleave(col(c, 6), col(c, 5), U, po.d, st));
  }
  // no stream sync: the pass's outputs are consumed in stream order
  passes.push_back(po);
  return SKS_OK;
}

// The scan's parameters for the m segments whose metadata sit in `arena` at the
// given word offsets (survivor / window counters zeroed there).
sks::ScanParams scan_params(const BuildState& S, const uint8_t* d_seq, const MetaArena& arena, size_t o_beg,
                            size_t o_end, size_t o_tp, size_t o_thr, size_t o_cap, size_t o_off, size_t o_cnt,
                            size_t o_win, uint32_t m, uint64_t n_tiles, size_t o_queue) {
  sks_ctx* c = S.c;
  sks::ScanParams p{};
  p.seq = d_seq;
  p.seg_begin = arena.ptr(o_beg);
  p.seg_end = arena.ptr(o_end);
  p.tile_prefix = arena.ptr(o_tp);
  p.n_seg = m;
  p.n_tiles = n_tiles;
  p.w = S.w;
  p.mask_lo = S.mask_lo;
  p.mask_hi = S.mask_hi;
  p.kconst = S.kconst;
  p.low_mask = S.dt.low_mask;
  p.high_mask = S.dt.rot > 32 ? (uint32_t)((1ull << (S.dt.rot - 32)) - 1) : 0u;
  p.dinv = S.dt.dinv;
  p.dlim = S.dt.lim;
  p.seg_thresh = arena.ptr(o_thr);
  p.out_key = reinterpret_cast<uint64_t*>(c->rec[0].ptr);
  p.out_val = reinterpret_cast<uint64_t*>(c->rec[1].ptr);
  p.out_hi = reinterpret_cast<uint64_t*>(c->rec[2].ptr);
  p.seg_out_off = arena.ptr(o_off);
  p.seg_out_cap = arena.ptr(o_cap);
  p.seg_count = reinterpret_cast<unsigned long long*>(arena.ptr(o_cnt));
  p.seg_windows = reinterpret_cast<unsigned long long*>(arena.ptr(o_win));
  static const bool static_tiles = getenv("SKS_SCAN_STATIC") != nullptr;
  p.tile_queue = static_tiles ? nullptr : reinterpret_cast<unsigned long long*>(arena.ptr(o_queue));
  return p;
}

constexpr int kFastFallback = -1;  // not an SKS status: take the general build

// One narrow bottom-s genome (kmer_set_from_fasta_file's shape, kmer_set.cpp:
// 54-68) whose candidates fit k_bottom_fused: the scan and the fused
// post-processing write the sketch set's own arrays, and the build's only host
// round trip is one read-back of (survivors, windows, size) at the end — instead
// of a count read-back, compaction, a device-wide sort and unique with a
// distinct-count read-back, select and a metadata upload.  A genome whose scan
// overflows the candidate region or that has fewer than s distinct candidates
// (both rare) returns kFastFallback and the general build runs instead.
int build_bottom_single(BuildState& S, const uint8_t* d_seq, const uint64_t* seg_off, uint64_t thresh,
                        uint64_t cap, sks_timings& tm, sks_sketch_set** out) {
  sks_ctx* c = S.c;
  hipStream_t st = c->stream;
  const uint64_t s = S.pol.param;
  const uint64_t n_tiles = sks::scan_tiles_for(seg_off[1] - seg_off[0]);
  SKS_HIP(c->rec[0].reserve(std::max<uint64_t>(cap, 1) * sizeof(uint64_t)));
  SKS_HIP(c->rec[1].reserve(std::max<uint64_t>(cap, 1) * sizeof(uint64_t)));
  const uint64_t slots = std::max<uint64_t>(std::min(s, cap), 1);
  MetaArena arena(c);
  const size_t o_beg = arena.add({seg_off[0]}), o_end = arena.add({seg_off[1]}), o_tp = arena.add({0, n_tiles}),
               o_thr = arena.add({thresh}), o_cap = arena.add({cap}), o_off = arena.add({0}),
               o_retry = arena.add({thresh != ~0ull ? 1ull : 0ull}), o_dst = arena.add({0, slots}),
               o_cnt = arena.add_zero(1), o_win = arena.add_zero(1), o_res = arena.add_zero(1),
               o_queue = arena.add_zero(1);
  if (o_win != o_cnt + 2 || o_res != o_win + 2) return sks::fail(SKS_E_HIP, "sks_sketch_build: arena layout");
  SKS_TRY(arena.upload());
  sks_sketch_set* set = new (std::nothrow) sks_sketch_set();
  if (!set) return sks::fail(SKS_E_NOMEM, "sks_sketch_build: out of memory");
  set->device = c->device;
  set->n = 1;
  int rc = alloc_u64(&set->d_data, slots);
  if (rc == SKS_OK) rc = alloc_u64(&set->d_starts, 1);
  if (rc == SKS_OK && dev_alloc(reinterpret_cast<void**>(&set->d_sizes), sizeof(uint32_t)) != hipSuccess)
    rc = sks::fail(SKS_E_HIP, "sks_sketch_build: device allocation failed");
  auto drop = [&]() {  // arrays still unused by the device or idle after a sync
    dev_release(set->d_data, slots * 8);
    dev_release(set->d_starts, 8);
    dev_release(set->d_sizes, 8);
    delete set;
  };
  if (rc != SKS_OK) {
    drop();
    return rc;
  }
  const sks::ScanParams p =
      scan_params(S, d_seq, arena, o_beg, o_end, o_tp, o_thr, o_cap, o_off, o_cnt, o_win, 1, n_tiles, o_queue);
  const sks::BitRuns runs = sks::bit_runs(S.mask_lo);
  const int kb = std::max(1, __builtin_popcountll(S.mask_lo));
  hipError_t e = hipEventRecord(c->ev_s0, st);
  if (e == hipSuccess) e = sks::launch_scan(p, sks::kModeBottom, S.pol.flavour, false, c->device, st, c->grid_override);
  if (e == hipSuccess) e = hipEventRecord(c->ev_s1, st);
  if (e == hipSuccess)
    e = sks::launch_bottom_fused(reinterpret_cast<uint64_t*>(c->rec[0].ptr), arena.ptr(o_off), arena.ptr(o_cnt),
                                 arena.ptr(o_retry), arena.ptr(o_dst), 1, cap, s, kb, runs, S.kconst,
                                 S.pol.flavour, set->d_data, arena.ptr(o_res), st, arena.ptr(o_cap), set->d_sizes,
                                 set->d_starts);
  if (e == hipSuccess) e = hipEventRecord(c->ev_end, st);
  uint64_t h[6] = {0, 0, 0, 0, 0, 0};  // survivors, -, windows, -, size, -
  if (e == hipSuccess) e = sks::pinned_d2h(h, arena.ptr(o_cnt), sizeof h, st);  // synchronises the stream
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(st);
    drop();
    return sks::fail(SKS_E_HIP, std::string("sks_sketch_build: ") + hipGetErrorString(e));
  }
  const uint64_t survivors = h[0], windows = h[2], size = h[4];
  if (survivors > cap || size == ~0ull || size == sks::kBottomOverflow || size > slots) {
    drop();
    return kFastFallback;
  }
  float ms = 0, tot = 0;
  (void)hipEventElapsedTime(&ms, c->ev_s0, c->ev_s1);
  (void)hipEventElapsedTime(&tot, c->ev_begin, c->ev_end);
  tm.scan_ms = ms;
  tm.scan_launches = n_tiles ? 1 : 0;
  tm.survivors = survivors;
  tm.windows = windows;
  tm.total_ms = tot;
  tm.post_ms = tot - ms;
  set->elem_words = 1;
  set->sizes = {(uint32_t)size};
  set->starts = {0};
  set->windows = {windows};
  set->window = S.w;
  set->mask[0] = S.mask_lo;
  set->mask[1] = S.mask_hi;
  set->policy = S.pol;
  c->last = tm;
  *out = set;
  return SKS_OK;
}

// Argument checks shared by sks_sketch_build and sks_kmer_list_build.
int validate_build(const char* fn, sks_ctx* c, const uint8_t* d_seq, uint64_t n_bytes,
                   const uint64_t* seg_off, uint32_t n_seg, int window, const uint64_t mask[2],
                   const sks_policy* policy) {
  const std::string f(fn);
  if (!c || !mask || !policy || (!seg_off && n_seg)) return sks::fail(SKS_E_ARG, f + ": null argument");
  if (window < 1 || window > 64)
    return sks::fail(SKS_E_ARG, f + ": window must be in [1, 64] (MAX_KMER_LENGTH)");
  if (policy->kind != SKS_FRAC_MOD && policy->kind != SKS_BOTTOM_S)
    return sks::fail(SKS_E_ARG, f + ": unknown policy kind");
  if (policy->flavour != 0 && policy->flavour != 1)
    return sks::fail(SKS_E_ARG, f + ": unknown hash flavour");
  if (policy->param == 0) return sks::fail(SKS_E_ARG, f + ": policy param must be > 0");
  {
    const int bits = 2 * window;
    uint64_t lo_allowed = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    uint64_t hi_allowed = bits <= 64 ? 0 : (bits >= 128 ? ~0ull : ((1ull << (bits - 64)) - 1));
    if ((mask[0] & ~lo_allowed) || (mask[1] & ~hi_allowed))
      return sks::fail(SKS_E_UNSUPPORTED,
                       f + ": mask has bits at or above 2*window (the reference's "
                       "generate_random_spaced_seed_mask never produces such masks)");
  }
  if (n_bytes && !d_seq) return sks::fail(SKS_E_ARG, f + ": null sequence");
  for (uint32_t g = 0; g < n_seg; ++g)
    if (seg_off[g] > seg_off[g + 1] || seg_off[g + 1] > n_bytes)
      return sks::fail(SKS_E_ARG, f + ": segment offsets must be non-decreasing and <= n_bytes");

  return SKS_OK;
}

}  // namespace

extern "C" {

int sks_sketch_build(sks_ctx* c, const uint8_t* d_seq, uint64_t n_bytes, const uint64_t* seg_off,
                     uint32_t n_seg, int window, const uint64_t mask[2], const sks_policy* policy,
                     sks_sketch_set** out) {
  if (!out) return sks::fail(SKS_E_ARG, "sks_sketch_build: null argument");
  *out = nullptr;
  SKS_TRY(validate_build("sks_sketch_build", c, d_seq, n_bytes, seg_off, n_seg, window, mask, policy));

  DeviceGuard guard(c->device);
  hipStream_t st = c->stream;
  BuildState S{c, window, window > 32, window > 32 ? 2 : 1, mask[0], mask[1], *policy,
               sks::fmh_const(mask[0], mask[1], window, policy->nonce, policy->flavour), {}};
  if (policy->kind == SKS_FRAC_MOD) S.dt = sks::make_div_test(policy->param);
  const bool bottom = policy->kind == SKS_BOTTOM_S;
  // bottom-s candidate margin: the first threshold keeps ~alpha*s windows, at
  // least 10 standard deviations above s for s >= 100 (a shortfall re-scans
  // that genome with a larger threshold).
  const double alpha = 1.0 + 10.0 / std::sqrt((double)policy->param) + 1.0 / (double)policy->param;

  sks_timings tm{};
  SKS_HIP(hipEventRecord(c->ev_begin, st));

  std::vector<uint64_t> thresh_g(n_seg, ~0ull), cap_g(n_seg), windows_g(n_seg, 0);
  std::vector<uint64_t> final_size(n_seg, ~0ull);
  for (uint32_t g = 0; g < n_seg; ++g) {
    const uint64_t L = seg_off[g + 1] - seg_off[g];
    double expect;
    if (!bottom) {
      expect = (double)L / (double)policy->param;
    } else {
      double want = alpha * (double)policy->param;
      if ((double)L <= want) {
        thresh_g[g] = ~0ull;
        expect = (double)L;
      } else {
        long double t = (long double)want / (long double)L * 18446744073709551616.0L;
        thresh_g[g] = t >= 18446744073709551615.0L ? ~0ull : (uint64_t)t;
        expect = want;
      }
    }
    double cap = expect + 6.0 * std::sqrt(expect) + 4096.0;
    cap_g[g] = (uint64_t)std::min<double>(cap, (double)L + 1.0);
  }

  // one narrow bottom-s genome: the single-round-trip path when its candidate
  // region fits the fused post-processing (8 standard deviations of the
  // candidate count above its mean, not the general margin, so the kernel runs
  // at the smaller register tile)
  if (bottom && !S.wide && n_seg == 1 && getenv("SKS_NO_FAST_BOTTOM") == nullptr) {
    const uint64_t L = seg_off[1] - seg_off[0];
    const double expect = std::min<double>((double)L, alpha * (double)policy->param);
    const uint64_t cap = std::min<uint64_t>(cap_g[0], (uint64_t)(expect + 8.0 * std::sqrt(expect) + 256.0));
    if (L > 0 && cap <= sks::bottom_fused_capacity()) {
      const int rc = build_bottom_single(S, d_seq, seg_off, thresh_g[0], cap, tm, out);
      if (rc != kFastFallback) return rc;
      tm = sks_timings{};
    }
  }

  std::vector<PassOut> passes;
  std::vector<uint32_t> pending(n_seg);
  std::iota(pending.begin(), pending.end(), 0);
  int guard_passes = 0;
  while (!pending.empty()) {
    if (++guard_passes > 64) {
      free_passes(passes);
      return sks::fail(SKS_E_HIP, "sks_sketch_build: selection did not converge");
    }
    const uint32_t m = (uint32_t)pending.size();
    std::vector<uint64_t> beg(m), end(m), tp(m + 1, 0), thr(m), cap(m), ooff(m);
    uint64_t total_cap = 0;
    for (uint32_t i = 0; i < m; ++i) {
      uint32_t g = pending[i];
      beg[i] = seg_off[g];
      end[i] = seg_off[g + 1];
      tp[i + 1] = tp[i] + sks::scan_tiles_for(end[i] - beg[i]);
      thr[i] = thresh_g[g];
      cap[i] = cap_g[g];
      ooff[i] = total_cap;
      total_cap += cap[i];
    }
    const uint64_t n_tiles = tp[m];
    for (int r = 0; r < (bottom && S.wide ? 3 : (bottom || S.wide ? 2 : 1)); ++r)
      SKS_HIP(c->rec[r].reserve(std::max<uint64_t>(total_cap, 1) * sizeof(uint64_t)));
    MetaArena arena(c);
    size_t o_beg = arena.add(beg), o_end = arena.add(end), o_tp = arena.add(tp),
           o_thr = arena.add(thr), o_cap = arena.add(cap), o_off = arena.add(ooff),
           o_cnt = arena.add_zero(m), o_win = arena.add_zero(m), o_queue = arena.add_zero(1);
    SKS_TRY(arena.upload());

    const sks::ScanParams p = scan_params(S, d_seq, arena, o_beg, o_end, o_tp, o_thr, o_cap, o_off, o_cnt, o_win,
                                          m, n_tiles, o_queue);

    SKS_HIP(hipEventRecord(c->ev_s0, st));
    SKS_HIP(sks::launch_scan(p, bottom ? sks::kModeBottom : sks::kModeFrac, policy->flavour,
                             S.wide, c->device, st, c->grid_override));
    SKS_HIP(hipEventRecord(c->ev_s1, st));
    tm.scan_launches += n_tiles ? 1 : 0;
    // survivor and window counts sit next to each other in the arena: one read-back
    if (o_win != o_cnt + m + 1) return sks::fail(SKS_E_HIP, "sks_sketch_build: arena layout");
    std::vector<uint64_t> cw(2 * (m + 1));
    SKS_HIP(sks::pinned_d2h(cw.data(), arena.ptr(o_cnt), cw.size() * sizeof(uint64_t), st));
    std::vector<uint64_t> counts(cw.begin(), cw.begin() + m), wins(cw.begin() + (m + 1), cw.begin() + (m + 1) + m);
    float ms = 0;
    SKS_HIP(hipEventElapsedTime(&ms, c->ev_s0, c->ev_s1));
    tm.scan_ms += ms;

    std::vector<uint32_t> ok, next;
    for (uint32_t i = 0; i < m; ++i) {
      tm.survivors += counts[i];
      if (counts[i] > cap[i]) {
        cap_g[pending[i]] = counts[i];
        next.push_back(pending[i]);
      } else {
        ok.push_back(i);
        windows_g[pending[i]] = wins[i];
      }
    }
    std::vector<uint32_t> retry_local;
    std::vector<uint64_t> fsz(m, ~0ull);
    int rc = post_process(S, pending, ooff, counts, thr, ok, passes, retry_local, fsz);
    if (rc != SKS_OK) {
      free_passes(passes);
      return rc;
    }
    for (uint32_t i : ok)
      if (fsz[i] != ~0ull) final_size[pending[i]] = fsz[i];
    for (uint32_t i : retry_local) {
      uint32_t g = pending[i];
      uint64_t t = thresh_g[g];
      thresh_g[g] = t > (~0ull >> 3) ? ~0ull : t * 8;
      uint64_t L = seg_off[g + 1] - seg_off[g];
      cap_g[g] = std::min<uint64_t>(L + 1, std::max<uint64_t>(cap_g[g], counts[i]) * 8 + 4096);
      next.push_back(g);
    }
    std::sort(next.begin(), next.end());
    pending.swap(next);
  }

  // assemble the final set in segment order
  sks_sketch_set* set = new (std::nothrow) sks_sketch_set();
  if (!set) {
    free_passes(passes);
    return sks::fail(SKS_E_NOMEM, "sks_sketch_build: out of memory");
  }
  set->device = c->device;
  set->elem_words = S.ew;
  set->n = n_seg;
  set->sizes.resize(n_seg);
  set->starts.resize(n_seg);
  set->windows = windows_g;
  set->window = window;
  set->mask[0] = mask[0];
  set->mask[1] = mask[1];
  set->policy = *policy;
  uint64_t total = 0;
  for (uint32_t g = 0; g < n_seg; ++g) {
    set->starts[g] = total;
    set->sizes[g] = (uint32_t)final_size[g];
    total += final_size[g];
  }
  int rc = SKS_OK;
  const bool single_in_order =
      passes.size() == 1 && passes[0].segs.size() == n_seg &&
      std::is_sorted(passes[0].segs.begin(), passes[0].segs.end());
  if (single_in_order) {
    set->d_data = passes[0].d;
    passes[0].d = nullptr;
  } else {
    rc = alloc_u64(&set->d_data, total * S.ew);
    for (size_t pi = 0; rc == SKS_OK && pi < passes.size(); ++pi) {
      const PassOut& po = passes[pi];
      const uint32_t k = (uint32_t)po.segs.size();
      if (k == 0) continue;
      std::vector<uint64_t> src(k + 1), dst(k + 1);
      uint64_t max_len = 0;
      for (uint32_t i = 0; i < k; ++i) {
        src[i] = po.off[i] * S.ew;
        dst[i] = set->starts[po.segs[i]] * S.ew;
        max_len = std::max(max_len, (po.off[i + 1] - po.off[i]) * S.ew);
      }
      // compact_regions reads len from dst_off[g+1]-dst_off[g]: run one segment at a time
      // via a per-segment CSR pair (dst, dst + len)
      for (uint32_t i = 0; i < k && rc == SKS_OK; ++i) {
        uint64_t len = (po.off[i + 1] - po.off[i]) * S.ew;
        if (!len) continue;
        if (hipMemcpyAsync(set->d_data + dst[i], po.d + src[i], len * sizeof(uint64_t),
                           hipMemcpyDeviceToDevice, st) != hipSuccess)
          rc = sks::fail(SKS_E_HIP, "sks_sketch_build: assembling copy failed");
      }
      (void)max_len;
    }
  }
  if (rc == SKS_OK) rc = alloc_u64(&set->d_starts, n_seg);
  if (rc == SKS_OK && dev_alloc(reinterpret_cast<void**>(&set->d_sizes),
                                std::max<uint32_t>(n_seg, 1) * sizeof(uint32_t)) != hipSuccess)
    rc = sks::fail(SKS_E_HIP, "sks_sketch_build: device allocation failed");
  if (rc == SKS_OK && n_seg) {
    if (sks::pinned_h2d(set->d_starts, set->starts.data(), n_seg * sizeof(uint64_t), st) !=
            hipSuccess ||
        sks::pinned_h2d(set->d_sizes, set->sizes.data(), n_seg * sizeof(uint32_t), st) != hipSuccess)
      rc = sks::fail(SKS_E_HIP, "sks_sketch_build: metadata upload failed");
  }
  if (rc == SKS_OK && hipEventRecord(c->ev_end, st) != hipSuccess)
    rc = sks::fail(SKS_E_HIP, "hipEventRecord failed");
  if (rc == SKS_OK && hipStreamSynchronize(st) != hipSuccess)
    rc = sks::fail(SKS_E_HIP, "hipStreamSynchronize failed");
  free_passes(passes);
  if (rc != SKS_OK) {
    sks_sketch_set_free(set);
    return rc;
  }
  float tot = 0;
  (void)hipEventElapsedTime(&tot, c->ev_begin, c->ev_end);
  tm.total_ms = tot;
  tm.post_ms = tot - tm.scan_ms;
  for (uint64_t wv : windows_g) tm.windows += wv;
  c->last = tm;
  *out = set;
  return SKS_OK;
}

int sks_sketch_set_free(sks_sketch_set* set) {
  if (!set) return SKS_OK;
  DeviceGuard g(set->device);
  // hipFree's contract: work queued on the arrays (any stream) completes before
  // they are reused; then they go to the block cache instead of being unmapped
  if (set->d_data || set->d_starts || set->d_sizes) (void)hipDeviceSynchronize();
  release_set_arrays(set, nullptr, false);
  delete set;
  return SKS_OK;
}

int sks_sketch_set_free_on_stream(sks_sketch_set* set, void* stream) {
  if (!set) return SKS_OK;
  DeviceGuard g(set->device);
  release_set_arrays(set, reinterpret_cast<hipStream_t>(stream), true);
  delete set;
  return SKS_OK;
}

uint32_t sks_sketch_set_num(const sks_sketch_set* set) { return set ? set->n : 0; }

int sks_sketch_set_elem_words(const sks_sketch_set* set) { return set ? set->elem_words : 0; }

int sks_sketch_set_sizes(const sks_sketch_set* set, uint32_t* sizes) {
  if (!set || !sizes) return sks::fail(SKS_E_ARG, "sks_sketch_set_sizes: null argument");
  std::copy(set->sizes.begin(), set->sizes.end(), sizes);
  return SKS_OK;
}

int sks_sketch_set_windows(const sks_sketch_set* set, uint64_t* windows) {
  if (!set || !windows) return sks::fail(SKS_E_ARG, "sks_sketch_set_windows: null argument");
  std::copy(set->windows.begin(), set->windows.end(), windows);
  return SKS_OK;
}

int sks_sketch_set_starts(const sks_sketch_set* set, uint64_t* starts) {
  if (!set || !starts) return sks::fail(SKS_E_ARG, "sks_sketch_set_starts: null argument");
  std::copy(set->starts.begin(), set->starts.end(), starts);
  return SKS_OK;
}

const uint64_t* sks_sketch_set_device_data(const sks_sketch_set* set) { return set ? set->d_data : nullptr; }
const uint64_t* sks_sketch_set_device_starts(const sks_sketch_set* set) { return set ? set->d_starts : nullptr; }
const uint32_t* sks_sketch_set_device_sizes(const sks_sketch_set* set) { return set ? set->d_sizes : nullptr; }

int sks_sketch_set_copy(const sks_sketch_set* set, uint32_t i, uint64_t* out) {
  if (!set) return sks::fail(SKS_E_ARG, "sks_sketch_set_copy: null set");
  if (i >= set->n) return sks::fail(SKS_E_ARG, "sks_sketch_set_copy: index out of range");
  if (!out && set->sizes[i]) return sks::fail(SKS_E_ARG, "sks_sketch_set_copy: null output");
  DeviceGuard g(set->device);
  uint64_t words = (uint64_t)set->sizes[i] * set->elem_words;
  if (words)
    SKS_HIP(hipMemcpy(out, set->d_data + set->starts[i] * set->elem_words, words * sizeof(uint64_t),
                      hipMemcpyDeviceToHost));
  return SKS_OK;
}

int sks_sketch_set_export(const sks_sketch_set* set, uint64_t* d_dst, uint64_t stride,
                          uint32_t* d_sizes) {
  if (!set || !d_dst || !d_sizes) return sks::fail(SKS_E_ARG, "sks_sketch_set_export: null argument");
  for (uint32_t s : set->sizes)
    if (s > stride) return sks::fail(SKS_E_ARG, "sks_sketch_set_export: stride smaller than a sketch");
  DeviceGuard g(set->device);
  SKS_HIP(sks::launch_export(set->d_data, set->d_starts, set->d_sizes, set->n, set->elem_words,
                             d_dst, stride, d_sizes, nullptr));
  SKS_HIP(hipStreamSynchronize(nullptr));
  return SKS_OK;
}

// ---- ordered k-mer lists (nucleotide_string_list_to_kmers) -----------------------------------

int sks_kmer_list_build(sks_ctx* c, const uint8_t* d_seq, uint64_t n_bytes, const uint64_t* seg_off,
                        uint32_t n_seg, int window, const uint64_t mask[2], const sks_policy* policy,
                        sks_kmer_list** out) {
  if (!out) return sks::fail(SKS_E_ARG, "sks_kmer_list_build: null argument");
  *out = nullptr;
  SKS_TRY(validate_build("sks_kmer_list_build", c, d_seq, n_bytes, seg_off, n_seg, window, mask,
                         policy));
  if (policy->kind != SKS_FRAC_MOD)
    return sks::fail(SKS_E_UNSUPPORTED,
                     "sks_kmer_list_build: lists take a per-k-mer predicate (SKS_FRAC_MOD); "
                     "bottom-s is a set selection");
  DeviceGuard guard(c->device);
  hipStream_t st = c->stream;
  const bool wide = window > 32;
  const sks::DivTest dt = sks::make_div_test(policy->param);
  std::vector<uint64_t> beg(n_seg), end(n_seg), tp(n_seg + 1, 0), cap(n_seg), ooff(n_seg);
  for (uint32_t g = 0; g < n_seg; ++g) {
    beg[g] = seg_off[g];
    end[g] = seg_off[g + 1];
    tp[g + 1] = tp[g] + sks::scan_tiles_for(end[g] - beg[g]);
    const double expect = (double)(end[g] - beg[g]) / (double)policy->param;
    cap[g] = (uint64_t)std::min<double>(expect + 6.0 * std::sqrt(expect) + 4096.0,
                                        (double)(end[g] - beg[g]) + 1.0);
  }
  std::vector<uint64_t> counts(n_seg, 0);
  for (int pass = 0; pass < 2; ++pass) {  // pass 2 only if a capacity estimate overflowed
    uint64_t total_cap = 0;
    for (uint32_t g = 0; g < n_seg; ++g) {
      ooff[g] = total_cap;
      total_cap += cap[g];
    }
    SKS_HIP(c->rec[0].reserve(std::max<uint64_t>(total_cap, 1) * sizeof(uint64_t)));
    MetaArena arena(c);
    size_t o_beg = arena.add(beg), o_end = arena.add(end), o_tp = arena.add(tp),
           o_cap = arena.add(cap), o_off = arena.add(ooff), o_cnt = arena.add_zero(n_seg),
           o_win = arena.add_zero(n_seg);
    SKS_TRY(arena.upload());
    sks::ScanParams p{};
    p.seq = d_seq;
    p.seg_begin = arena.ptr(o_beg);
    p.seg_end = arena.ptr(o_end);
    p.tile_prefix = arena.ptr(o_tp);
    p.n_seg = n_seg;
    p.n_tiles = tp[n_seg];
    p.w = window;
    p.mask_lo = mask[0];
    p.mask_hi = mask[1];
    p.kconst = sks::fmh_const(mask[0], mask[1], window, policy->nonce, policy->flavour);
    p.low_mask = dt.low_mask;
    p.high_mask = dt.rot > 32 ? (uint32_t)((1ull << (dt.rot - 32)) - 1) : 0u;
    p.dinv = dt.dinv;
    p.dlim = dt.lim;
    p.seg_thresh = arena.ptr(o_cap);  // unused in list mode
    p.out_key = reinterpret_cast<uint64_t*>(c->rec[0].ptr);
    p.seg_out_off = arena.ptr(o_off);
    p.seg_out_cap = arena.ptr(o_cap);
    p.seg_count = reinterpret_cast<unsigned long long*>(arena.ptr(o_cnt));
    p.seg_windows = reinterpret_cast<unsigned long long*>(arena.ptr(o_win));
    SKS_HIP(sks::launch_scan(p, sks::kModeList, policy->flavour, wide, c->device, st,
                             c->grid_override));
    SKS_HIP(sks::pinned_d2h(counts.data(), p.seg_count, n_seg * sizeof(uint64_t), st));
    bool overflow = false;
    for (uint32_t g = 0; g < n_seg; ++g)
      if (counts[g] > cap[g]) {
        overflow = true;
        cap[g] = counts[g];
      }
    if (!overflow) break;
    if (pass == 1) return sks::fail(SKS_E_HIP, "sks_kmer_list_build: survivor count changed between passes");
  }
  // dense positions (segments in stream order), then one sort: stream order
  std::vector<uint64_t> csr = prefix(counts);
  const uint64_t T = csr[n_seg];
  uint64_t max_len = 0;
  for (uint64_t v : counts) max_len = std::max(max_len, v);
  sks_kmer_list* kl = new (std::nothrow) sks_kmer_list();
  if (!kl) return sks::fail(SKS_E_NOMEM, "sks_kmer_list_build: out of memory");
  kl->device = c->device;
  kl->n = n_seg;
  kl->total = T;
  kl->counts = counts;
  int rc = alloc_u64(&kl->d_pos, T);
  if (rc == SKS_OK) rc = alloc_u64(&kl->d_bits, 4 * T);
  if (rc == SKS_OK) rc = reserve_cols(c, {0}, T + 1);
  MetaArena arena(c);
  size_t o_src = arena.add(ooff), o_csr = arena.add(csr), o_beg = arena.add(beg);
  if (rc == SKS_OK) rc = arena.upload();
  hipError_t e = hipSuccess;
  if (rc == SKS_OK && T) {
    e = sks::compact_regions(reinterpret_cast<uint64_t*>(c->rec[0].ptr), col(c, 0), arena.ptr(o_src),
                             arena.ptr(o_csr), n_seg, max_len, st);
    if (e == hipSuccess)
      e = sks::seg_sort_keys(col(c, 0), kl->d_pos, T, {0, T}, nullptr, end_bit_of(n_bytes), c->tmp, st);
    if (e == hipSuccess)
      e = sks::launch_materialise(d_seq, arena.ptr(o_beg), n_seg, kl->d_pos, T, window, mask[0],
                                  mask[1], kl->d_bits, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = sks::fail(SKS_E_HIP, std::string("sks_kmer_list_build: ") + hipGetErrorString(e));
  }
  if (rc != SKS_OK) {
    sks_kmer_list_free(kl);
    return rc;
  }
  *out = kl;
  return SKS_OK;
}

int sks_kmer_list_free(sks_kmer_list* kl) {
  if (!kl) return SKS_OK;
  DeviceGuard g(kl->device);
  if (kl->d_pos) (void)hipFree(kl->d_pos);
  if (kl->d_bits) (void)hipFree(kl->d_bits);
  delete kl;
  return SKS_OK;
}

uint64_t sks_kmer_list_total(const sks_kmer_list* kl) { return kl ? kl->total : 0; }

int sks_kmer_list_counts(const sks_kmer_list* kl, uint64_t* counts) {
  if (!kl || (!counts && kl->n)) return sks::fail(SKS_E_ARG, "sks_kmer_list_counts: null argument");
  std::copy(kl->counts.begin(), kl->counts.end(), counts);
  return SKS_OK;
}

const uint64_t* sks_kmer_list_device_positions(const sks_kmer_list* kl) { return kl ? kl->d_pos : nullptr; }
const uint64_t* sks_kmer_list_device_bits(const sks_kmer_list* kl) { return kl ? kl->d_bits : nullptr; }

int sks_kmer_list_copy(const sks_kmer_list* kl, uint64_t* positions, uint64_t* bits) {
  if (!kl) return sks::fail(SKS_E_ARG, "sks_kmer_list_copy: null list");
  DeviceGuard g(kl->device);
  if (positions && kl->total)
    SKS_HIP(hipMemcpy(positions, kl->d_pos, kl->total * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (bits && kl->total)
    SKS_HIP(hipMemcpy(bits, kl->d_bits, kl->total * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return SKS_OK;
}

// Group bounds fixed by the mask alone (no sample of the sketches): a masked
// canonical k-mer of random sequence is min(F & M, R & M) of two near-uniform
// values over the mask's 2k bits, so its packed value (the mask bits gathered)
// has CDF 1 - (1 - x)^2 and the g/G quantile is x = 1 - sqrt(1 - g/G); the
// bound is that packed value scattered back onto the mask bits (a pdep).  Any
// non-decreasing bounds give exact counts (layout.hip): these only balance the
// groups, and need no device pass and no exchange between ranks.
int sks_join_layout_bounds_for_mask(const uint64_t mask[2], uint32_t log_b, int elem_words, uint64_t* bounds) {
  if (!mask || !bounds) return sks::fail(SKS_E_ARG, "sks_join_layout_bounds_for_mask: null argument");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (elem_words == 1 && mask[1]) return sks::fail(SKS_E_ARG, "sks_join_layout_bounds_for_mask: a 128-bit mask "
                                                               "needs elem_words = 2");
  const uint32_t G = sks_join_layout_groups(log_b);
  const int P = __builtin_popcountll(mask[0]) + __builtin_popcountll(mask[1]);
  auto pdep = [&](uint64_t vlo, uint64_t vhi, uint64_t* lo, uint64_t* hi) {
    *lo = *hi = 0;
    int j = 0;  // packed bit j -> the j-th set bit of the mask
    for (int b = 0; b < 128; ++b) {
      if (!((b < 64 ? mask[0] >> b : mask[1] >> (b - 64)) & 1)) continue;
      const uint64_t bit = j < 64 ? (vlo >> j) & 1 : (vhi >> (j - 64)) & 1;
      if (bit) {
        if (b < 64) *lo |= 1ull << b;
        else *hi |= 1ull << (b - 64);
      }
      ++j;
    }
  };
  for (uint32_t g = 0; g <= G; ++g) {
    uint64_t lo = 0, hi = 0;
    if (g == G) {
      lo = ~0ull;
      hi = elem_words == 2 ? ~0ull : 0;
    } else if (g > 0 && P > 0) {
      const long double x = 1.0L - std::sqrt(1.0L - (long double)g / (long double)G);
      uint64_t vlo = 0, vhi = 0;
      if (P <= 64) {
        const long double v = std::ldexp(x, P);
        vlo = v >= 18446744073709551615.0L ? (P == 64 ? ~0ull : (1ull << P) - 1) : (uint64_t)v;
      } else {
        const long double v = std::ldexp(x, P - 64);
        vhi = (uint64_t)std::floor(v);
        vlo = (uint64_t)std::ldexp(v - std::floor(v), 64);
      }
      pdep(vlo, vhi, &lo, &hi);
    }
    bounds[(size_t)g * elem_words] = lo;
    if (elem_words == 2) bounds[(size_t)g * 2 + 1] = hi;
  }
  return SKS_OK;
}

int sks_windows_dense_row_words(int window) { return window > 32 ? 4 : 3; }

int sks_windows_dense(sks_ctx* c, const uint8_t* d_seq, uint64_t n_bytes, uint64_t first, uint64_t n_windows,
                      int window, const uint64_t mask[2], uint64_t* d_rows, uint64_t* d_valid) {
  if (!c || !mask) return sks::fail(SKS_E_ARG, "sks_windows_dense: null argument");
  if (window < 1 || window > 64) return sks::fail(SKS_E_ARG, "sks_windows_dense: window must be 1..64");
  if (first > n_bytes) return sks::fail(SKS_E_ARG, "sks_windows_dense: first beyond the buffer");
  if (n_windows == 0) return SKS_OK;
  if (!d_seq || !d_rows || !d_valid) return sks::fail(SKS_E_ARG, "sks_windows_dense: null buffer");
  DeviceGuard g(c->device);
  SKS_HIP(sks::launch_windows_dense(d_seq, n_bytes, first, n_windows, window, mask[0], mask[1], d_rows, d_valid,
                                    c->stream));
  return SKS_OK;
}

// ---- intersections ----------------------------------------------------------------------------

int sks_intersect_pairs(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts,
                        const uint32_t* d_sizes, int elem_words, const int32_t* d_a,
                        const int32_t* d_b, uint64_t n_pairs, int32_t* d_out) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_intersect_pairs: null ctx");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (n_pairs && (!d_starts || !d_sizes || !d_a || !d_b || !d_out))
    return sks::fail(SKS_E_ARG, "sks_intersect_pairs: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  SKS_HIP(sks::launch_intersect_pairs(d_data, d_starts, d_sizes, elem_words, d_a, d_b, n_pairs,
                                      d_out, c->stream));
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_intersect_all(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts,
                      const uint32_t* d_sizes, int elem_words, uint32_t n, uint32_t row_begin,
                      uint32_t row_end, int32_t* d_out) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_intersect_all: null ctx");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (row_begin > row_end || row_end > n) return sks::fail(SKS_E_ARG, "sks_intersect_all: bad row range");
  if (row_end > row_begin && (!d_starts || !d_sizes || !d_out))
    return sks::fail(SKS_E_ARG, "sks_intersect_all: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  bool done = false;
  if (c->intersect_algo != sks::kIntersectGlobal)
    SKS_HIP(sks::launch_intersect_tiled(d_data, d_starts, d_sizes, n, false, row_begin, row_end, 0, 0,
                                        d_out, c->iwork, c->stream, &done, c->intersect_algo, elem_words,
                                        c->join_check));
  if (!done)
    SKS_HIP(sks::launch_intersect_all_global(d_data, d_starts, d_sizes, elem_words, n, row_begin,
                                             row_end, d_out, c->stream));
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

uint64_t sks_intersect_sym_tiles(uint32_t n) { return sks::intersect_sym_tiles(n); }

int sks_intersect_sym(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts,
                      const uint32_t* d_sizes, int elem_words, uint32_t n, uint64_t tile_begin,
                      uint64_t tile_end, int32_t* d_out) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_intersect_sym: null ctx");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (tile_begin > tile_end) return sks::fail(SKS_E_ARG, "sks_intersect_sym: bad tile range");
  if (n && (!d_starts || !d_sizes || !d_out)) return sks::fail(SKS_E_ARG, "sks_intersect_sym: null argument");
  DeviceGuard g(c->device);
  const uint64_t all = sks::intersect_sym_tiles(n);
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  bool done = false;
  if (c->intersect_algo != sks::kIntersectGlobal)
    SKS_HIP(sks::launch_intersect_tiled(d_data, d_starts, d_sizes, n, true, 0, n, tile_begin,
                                        tile_end, d_out, c->iwork, c->stream, &done,
                                        c->intersect_algo, elem_words, c->join_check));
  if (!done) {
    if (tile_begin != 0 || tile_end < all)
      return sks::fail(SKS_E_UNSUPPORTED,
                       "sks_intersect_sym: partial tile ranges need sketches without extreme "
                       "value skew; use sks_intersect_all row blocks");
    SKS_HIP(sks::launch_intersect_all_global(d_data, d_starts, d_sizes, elem_words, n, 0, n, d_out,
                                             c->stream));
  }
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_sketch_union(sks_ctx* c, const uint64_t* d_in, uint64_t n, uint64_t* d_out,
                     uint64_t* n_out) {
  if (!c || !n_out) return sks::fail(SKS_E_ARG, "sks_sketch_union: null argument");
  if (n && (!d_in || !d_out)) return sks::fail(SKS_E_ARG, "sks_sketch_union: null argument");
  if (n >= (1ull << 32)) return sks::fail(SKS_E_UNSUPPORTED, "sks_sketch_union: n >= 2^32");
  DeviceGuard g(c->device);
  SKS_HIP(sks::sort_unique_u64(d_in, n, d_out, n_out, c->iwork, c->stream));
  return SKS_OK;
}

int sks_sketch_union_wide(sks_ctx* c, const uint64_t* d_in, uint64_t n, uint64_t* d_out,
                          uint64_t* n_out) {
  if (!c || !n_out) return sks::fail(SKS_E_ARG, "sks_sketch_union_wide: null argument");
  if (n && (!d_in || !d_out)) return sks::fail(SKS_E_ARG, "sks_sketch_union_wide: null argument");
  if (n >= (1ull << 32)) return sks::fail(SKS_E_UNSUPPORTED, "sks_sketch_union_wide: n >= 2^32");
  if ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out)) & 15)
    return sks::fail(SKS_E_ARG, "sks_sketch_union_wide: buffers must be 16-byte aligned");
  DeviceGuard g(c->device);
  SKS_HIP(sks::sort_unique_u128(d_in, n, d_out, n_out, c->iwork, c->stream));
  return SKS_OK;
}

uint32_t sks_join_layout_log_b(uint32_t max_sketch_size) { return sks::join_log_b(max_sketch_size); }
uint32_t sks_join_layout_capacity(void) { return sks::join_cap(); }
uint32_t sks_join_layout_groups(uint32_t log_b) { return sks::join_layout_groups(log_b); }
uint32_t sks_join_layout_boff_words(uint32_t log_b) { return log_b > 14 ? 0u : sks::join_layout_boff_words(log_b); }

int sks_join_layout_bounds(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts,
                           const uint32_t* d_sizes, int elem_words, uint32_t n, uint32_t log_b,
                           uint64_t* d_bounds) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_join_layout_bounds: null ctx");
  if (log_b > 14) return sks::fail(SKS_E_ARG, "sks_join_layout_bounds: log_b > 14");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (!d_bounds || (n && (!d_starts || !d_sizes))) return sks::fail(SKS_E_ARG, "sks_join_layout_bounds: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(sks::join_layout_bounds(d_data, d_starts, d_sizes, n, log_b, elem_words, d_bounds, c->stream));
  return SKS_OK;
}

int sks_join_layout_build(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts,
                          const uint32_t* d_sizes, int elem_words, uint32_t n, uint64_t total_hint,
                          uint32_t log_b, const uint64_t* d_bounds, uint64_t* d_out_vals,
                          uint64_t* d_out_masks, uint32_t* d_out_boff, uint64_t* d_out_bstart,
                          uint32_t* max_block_bucket) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_join_layout_build: null ctx");
  if (log_b > 14) return sks::fail(SKS_E_ARG, "sks_join_layout_build: log_b > 14");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (!d_out_bstart || (n && (!d_starts || !d_sizes || !d_out_boff)))
    return sks::fail(SKS_E_ARG, "sks_join_layout_build: null argument");
  DeviceGuard g(c->device);
  uint64_t total = total_hint;
  if (n && total == UINT64_MAX) {  // unknown: read the sizes back (waits for the stream)
    std::vector<uint32_t> h_sizes(n);
    SKS_HIP(sks::pinned_d2h(h_sizes.data(), d_sizes, n * sizeof(uint32_t), c->stream));
    total = 0;
    for (uint32_t v : h_sizes) total += v;
  }
  if (!n) total = 0;
  // bucket starts are u32: the layout must hold < 2^32 elements
  if (total >= (1ull << 32))
    return sks::fail(SKS_E_UNSUPPORTED, "sks_join_layout_build: >= 2^32 elements in one layout");
  const size_t o_stat = (sks::join_layout_temp_bytes(n, log_b, elem_words) + 15) & ~(size_t)15;
  SKS_HIP(c->iwork.reserve(o_stat + 16));
  char* w = static_cast<char*>(c->iwork.ptr);
  uint32_t* stat = reinterpret_cast<uint32_t*>(w + o_stat);
  SKS_HIP(hipMemsetAsync(stat, 0, 8, c->stream));
  c->layout_stat = stat;
  if (n == 0) {
    SKS_HIP(hipMemsetAsync(d_out_bstart, 0, 8, c->stream));
  } else {
    SKS_HIP(sks::join_layout_build(d_data, d_starts, d_sizes, n, log_b, elem_words, d_bounds, w, d_out_vals,
                                   d_out_masks, d_out_boff, d_out_bstart, stat, c->join_check, c->stream, nullptr,
                                   c->layout_blocks_hint));
  }
  if (max_block_bucket) {  // NULL: no read-back, the call does not wait for the build
    uint32_t h[2] = {0, 0};
    SKS_HIP(sks::pinned_d2h(h, stat, 8, c->stream));
    *max_block_bucket = h[1] ? UINT32_MAX : h[0];
  }
  return SKS_OK;
}

int sks_join_layout_stat_copy(sks_ctx* c, uint32_t* d_dst) {
  if (!c || !d_dst) return sks::fail(SKS_E_ARG, "sks_join_layout_stat_copy: null argument");
  if (!c->layout_stat) return sks::fail(SKS_E_ARG, "sks_join_layout_stat_copy: no layout built on this context");
  DeviceGuard g(c->device);
  SKS_HIP(hipMemcpyAsync(d_dst, c->layout_stat, 8, hipMemcpyDeviceToDevice, c->stream));
  return SKS_OK;
}

int sks_intersect_sym_layout(sks_ctx* c, uint32_t n, uint32_t log_b, int elem_words, const uint64_t* d_vals,
                             const uint64_t* d_masks, const uint32_t* d_boff, const uint64_t* d_bstart,
                             uint64_t tile_begin, uint64_t tile_end, int32_t* d_out) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_intersect_sym_layout: null ctx");
  if (log_b > 14) return sks::fail(SKS_E_ARG, "sks_intersect_sym_layout: log_b > 14");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (tile_begin > tile_end) return sks::fail(SKS_E_ARG, "sks_intersect_sym_layout: bad tile range");
  if (n && (!d_boff || !d_bstart || !d_out))
    return sks::fail(SKS_E_ARG, "sks_intersect_sym_layout: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  SKS_HIP(hipMemsetAsync(d_out, 0, (uint64_t)n * n * sizeof(int32_t), c->stream));
  if (n) {
    const sks::JoinLayout L{d_vals, d_masks, d_boff, d_bstart};
    SKS_HIP(sks::join_launch(L, 0, L, 0, n, log_b, elem_words, true, 0, n, tile_begin, tile_end, nullptr, false,
                             d_out, c->join_check, c->stream));
  }
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_intersect_layout_tiles(sks_ctx* c, uint32_t n, uint32_t log_b, int elem_words, const uint64_t* d_vals,
                               const uint64_t* d_masks, const uint32_t* d_boff, const uint64_t* d_bstart,
                               uint32_t blk0, const uint32_t* d_tiles, uint64_t tile_begin,
                               uint64_t tile_end, int packed, int32_t* d_out) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_intersect_layout_tiles: null ctx");
  if (log_b > 14) return sks::fail(SKS_E_ARG, "sks_intersect_layout_tiles: log_b > 14");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (tile_begin > tile_end) return sks::fail(SKS_E_ARG, "sks_intersect_layout_tiles: bad tile range");
  if (!d_tiles && tile_end > sks::intersect_sym_tiles(n))
    return sks::fail(SKS_E_ARG, "sks_intersect_layout_tiles: tile range beyond the upper triangle");
  // the upper-triangle range starts at global block 0: a layout whose block 0
  // is another block holds only part of it (a tile list names its blocks)
  if (!d_tiles && blk0 != 0 && tile_end > tile_begin)
    return sks::fail(SKS_E_ARG, "sks_intersect_layout_tiles: a tile range needs blk0 = 0 (pass a tile list)");
  if (tile_end > tile_begin && (!d_boff || !d_bstart || !d_out))
    return sks::fail(SKS_E_ARG, "sks_intersect_layout_tiles: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  if (n && tile_end > tile_begin) {
    const sks::JoinLayout L{d_vals, d_masks, d_boff, d_bstart};
    SKS_HIP(sks::join_launch(L, 0u - blk0, L, 0u - blk0, n, log_b, elem_words, true, 0, n, tile_begin, tile_end,
                             d_tiles, packed != 0, d_out, c->join_check, c->stream));
  }
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_intersect_layout_pair_tiles(sks_ctx* c, uint32_t n, uint32_t log_b, int elem_words,
                                    const uint64_t* d_rvals, const uint64_t* d_rmasks, const uint32_t* d_rboff,
                                    const uint64_t* d_rbstart, uint32_t r_blk0, const uint64_t* d_cvals,
                                    const uint64_t* d_cmasks, const uint32_t* d_cboff, const uint64_t* d_cbstart,
                                    uint32_t c_blk0, const uint32_t* d_tiles, uint64_t tile_begin,
                                    uint64_t tile_end, int packed, int32_t* d_out) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_intersect_layout_pair_tiles: null ctx");
  if (log_b > 14) return sks::fail(SKS_E_ARG, "sks_intersect_layout_pair_tiles: log_b > 14");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (tile_begin > tile_end) return sks::fail(SKS_E_ARG, "sks_intersect_layout_pair_tiles: bad tile range");
  if (tile_end > tile_begin && (!d_tiles || !d_rboff || !d_rbstart || !d_cboff || !d_cbstart || !d_out))
    return sks::fail(SKS_E_ARG, "sks_intersect_layout_pair_tiles: null argument (a tile list is required)");
  DeviceGuard g(c->device);
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  if (n && tile_end > tile_begin) {
    const sks::JoinLayout R{d_rvals, d_rmasks, d_rboff, d_rbstart}, C{d_cvals, d_cmasks, d_cboff, d_cbstart};
    SKS_HIP(sks::join_launch(R, 0u - r_blk0, C, 0u - c_blk0, n, log_b, elem_words, true, 0, n, tile_begin,
                             tile_end, d_tiles, packed != 0, d_out, c->join_check, c->stream));
  }
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_intersect_layout_ani(sks_ctx* c, uint32_t n, uint32_t log_b, int elem_words, const uint64_t* d_rvals,
                             const uint64_t* d_rmasks, const uint32_t* d_rboff, const uint64_t* d_rbstart,
                             uint32_t r_blk0, const uint64_t* d_cvals, const uint64_t* d_cmasks,
                             const uint32_t* d_cboff, const uint64_t* d_cbstart, uint32_t c_blk0,
                             const uint32_t* d_tiles, uint64_t tile_begin, uint64_t tile_end, int packed,
                             int32_t* d_out, const int32_t* d_sizes, int kmer_num_ones, double* ani) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_intersect_layout_ani: null ctx");
  if (log_b > 14) return sks::fail(SKS_E_ARG, "sks_intersect_layout_ani: log_b > 14");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (kmer_num_ones <= 0) return sks::fail(SKS_E_ARG, "sks_intersect_layout_ani: kmer_num_ones must be positive");
  if (tile_begin > tile_end) return sks::fail(SKS_E_ARG, "sks_intersect_layout_ani: bad tile range");
  if (!d_tiles && tile_end > sks::intersect_sym_tiles(n))
    return sks::fail(SKS_E_ARG, "sks_intersect_layout_ani: tile range beyond the upper triangle");
  if (!d_tiles && tile_end > tile_begin && (r_blk0 != 0 || c_blk0 != 0 || d_rvals != d_cvals))
    return sks::fail(SKS_E_ARG, "sks_intersect_layout_ani: a tile range needs one layout with blk0 = 0 "
                                "(pass a tile list)");
  if (tile_end > tile_begin &&
      (!d_rboff || !d_rbstart || !d_cboff || !d_cbstart || !d_out || !d_sizes || !ani))
    return sks::fail(SKS_E_ARG, "sks_intersect_layout_ani: null argument");
  DeviceGuard g(c->device);
  // the ANI matrix may be host memory: the kernel needs its device-side address
  double* d_ani = ani;
  if (tile_end > tile_begin) SKS_TRY(device_view_of_ani(ani, &d_ani, "sks_intersect_layout_ani"));
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  if (n && tile_end > tile_begin) {
    const uint64_t nt = tile_end - tile_begin;
    SKS_HIP(c->tdone.reserve(nt * sizeof(uint32_t)));
    SKS_HIP(hipMemsetAsync(c->tdone.ptr, 0, nt * sizeof(uint32_t), c->stream));
    const sks::JoinLayout R{d_rvals, d_rmasks, d_rboff, d_rbstart}, C{d_cvals, d_cmasks, d_cboff, d_cbstart};
    sks::JoinAni A{d_ani, d_sizes, kmer_num_ones, static_cast<uint32_t*>(c->tdone.ptr)};
    if (c->root_k == kmer_num_ones) {  // the context's table (sks_ctx_ani_table), if for this k
      A.root = static_cast<const double*>(c->root.ptr);
      A.root_size = c->root_size;
    }
    SKS_HIP(sks::join_launch(R, 0u - r_blk0, C, 0u - c_blk0, n, log_b, elem_words, true, 0, n, tile_begin,
                             tile_end, d_tiles, packed != 0, d_out, c->join_check, c->stream, &A));
  }
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_all_pairs_ani(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts, const uint32_t* d_sizes,
                      int elem_words, uint32_t n, uint32_t max_size, uint64_t total, int kmer_num_ones,
                      double* ani, int32_t* d_counts, uint32_t* d_status) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_all_pairs_ani: null ctx");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (ani && kmer_num_ones <= 0) return sks::fail(SKS_E_ARG, "sks_all_pairs_ani: kmer_num_ones must be positive");
  if (n && (!d_starts || !d_sizes)) return sks::fail(SKS_E_ARG, "sks_all_pairs_ani: null argument");
  if (total >= (1ull << 32)) return sks::fail(SKS_E_UNSUPPORTED, "sks_all_pairs_ani: >= 2^32 elements");
  DeviceGuard g(c->device);
  double* d_ani = ani;
  if (ani && n) SKS_TRY(device_view_of_ani(ani, &d_ani, "sks_all_pairs_ani"));
  if (n == 0) {
    if (d_status) SKS_HIP(hipMemsetAsync(d_status, 0, 8, c->stream));
    SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
    SKS_HIP(hipEventRecord(c->ev_end, c->stream));
    return SKS_OK;
  }
  // one layout of all n sketches (context scratch), then every upper-triangle
  // tile in one join launch: packed counts and, when asked, the fused ANI
  const uint32_t log_b = sks::join_log_b(std::max<uint32_t>(max_size, 1));
  const uint32_t nb = (n + 63) / 64;
  const uint64_t T = sks::intersect_sym_tiles(n);
  const uint64_t tot = std::max<uint64_t>(total, 1);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_vals = 0, o_masks = al(o_vals + tot * 8 * elem_words), o_boff = al(o_masks + tot * 8);
  const size_t o_bst = al(o_boff + (size_t)nb * sks::join_layout_boff_words(log_b) * 4);
  const size_t o_stat = al(o_bst + (size_t)(nb + 1) * 8);
  const size_t o_cnt = al(o_stat + 16);
  const size_t o_tmp = al(o_cnt + (d_counts ? 0 : (size_t)T * 4096 * 4));
  const size_t need = o_tmp + sks::join_layout_temp_bytes(n, log_b, elem_words) + 256;
  SKS_HIP(c->lay.reserve(need));
  SKS_HIP(c->tdone.reserve(T * sizeof(uint32_t)));
  char* w = static_cast<char*>(c->lay.ptr);
  uint64_t* vals = reinterpret_cast<uint64_t*>(w + o_vals);
  uint64_t* masks = reinterpret_cast<uint64_t*>(w + o_masks);
  uint32_t* boff = reinterpret_cast<uint32_t*>(w + o_boff);
  uint64_t* bst = reinterpret_cast<uint64_t*>(w + o_bst);
  // the build's status words go straight to the caller's d_status
  uint32_t* stat = d_status ? d_status : reinterpret_cast<uint32_t*>(w + o_stat);
  int32_t* cnt = d_counts ? d_counts : reinterpret_cast<int32_t*>(w + o_cnt);
  // the status words, the count tiles and the tiles' finisher counters are
  // cleared by the build's second launch (no memsets of their own)
  const sks::ZeroSpans zs{{stat, reinterpret_cast<uint32_t*>(cnt), ani ? static_cast<uint32_t*>(c->tdone.ptr) : nullptr},
                          {2, T * 4096, ani ? T : 0}};
  SKS_HIP(sks::join_layout_build(d_data, d_starts, d_sizes, n, log_b, elem_words, nullptr, w + o_tmp, vals, masks,
                                 boff, bst, stat, c->join_check, c->stream, &zs));
  const sks::JoinLayout L{vals, masks, boff, bst};
  sks::JoinAni A{d_ani, reinterpret_cast<const int32_t*>(d_sizes), kmer_num_ones,
                 static_cast<uint32_t*>(c->tdone.ptr)};
  if (ani) {  // bottom-s sets all hold max_size elements: their ANI comes from the table
    SKS_TRY(sks_ctx_ani_table(c, max_size, kmer_num_ones));
    if (c->root_k == kmer_num_ones) {
      A.root = static_cast<const double*>(c->root.ptr);
      A.root_size = c->root_size;
    }
  }
  // sks_ctx_last_intersect_ms: the join launch alone (the layout build before it
  // is the call's fixed part)
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  SKS_HIP(sks::join_launch(L, 0, L, 0, n, log_b, elem_words, true, 0, n, 0, T, nullptr, true, cnt, c->join_check,
                           c->stream, ani ? &A : nullptr));
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_layout_tiles_ani(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts, const uint32_t* d_sizes,
                         int elem_words, uint32_t n, uint64_t total, uint32_t log_b, const uint64_t* d_bounds,
                         uint32_t blocks_hint, uint32_t blk0, const uint32_t* d_tiles, uint64_t n_tiles,
                         uint32_t n_global, const int32_t* d_sizes_global, int kmer_num_ones, double* ani,
                         int32_t* d_counts, uint32_t* d_status) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_layout_tiles_ani: null ctx");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (ani && kmer_num_ones <= 0) return sks::fail(SKS_E_ARG, "sks_layout_tiles_ani: kmer_num_ones must be positive");
  if (log_b > sks_join_layout_log_b(~0u)) return sks::fail(SKS_E_ARG, "sks_layout_tiles_ani: log_b too large");
  if (n_tiles && (!d_tiles || !d_counts || (ani && !d_sizes_global)))
    return sks::fail(SKS_E_ARG, "sks_layout_tiles_ani: null argument");
  if (n && (!d_starts || !d_sizes)) return sks::fail(SKS_E_ARG, "sks_layout_tiles_ani: null argument");
  if (total >= (1ull << 32)) return sks::fail(SKS_E_UNSUPPORTED, "sks_layout_tiles_ani: >= 2^32 elements");
  DeviceGuard g(c->device);
  double* d_ani = ani;
  if (ani && n_tiles) SKS_TRY(device_view_of_ani(ani, &d_ani, "sks_layout_tiles_ani"));
  if (n == 0 || n_tiles == 0) {
    if (d_status) SKS_HIP(hipMemsetAsync(d_status, 0, 8, c->stream));
    if (n_tiles) SKS_HIP(hipMemsetAsync(d_counts, 0, n_tiles * 4096 * 4, c->stream));
    SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
    SKS_HIP(hipEventRecord(c->ev_end, c->stream));
    return SKS_OK;
  }
  // the layout in context scratch, as sks_all_pairs_ani; its second launch
  // clears the caller's count tiles, the tiles' finisher counters and the
  // status words, so the whole call is four launches and no memset
  const uint32_t nb = (n + 63) / 64;
  const uint64_t tot = std::max<uint64_t>(total, 1);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_vals = 0, o_masks = al(o_vals + tot * 8 * elem_words), o_boff = al(o_masks + tot * 8);
  const size_t o_bst = al(o_boff + (size_t)nb * sks::join_layout_boff_words(log_b) * 4);
  const size_t o_stat = al(o_bst + (size_t)(nb + 1) * 8);
  const size_t o_tmp = al(o_stat + 16);
  const size_t need = o_tmp + sks::join_layout_temp_bytes(n, log_b, elem_words) + 256;
  SKS_HIP(c->lay.reserve(need));
  SKS_HIP(c->tdone.reserve(n_tiles * sizeof(uint32_t)));
  char* w = static_cast<char*>(c->lay.ptr);
  uint64_t* vals = reinterpret_cast<uint64_t*>(w + o_vals);
  uint64_t* masks = reinterpret_cast<uint64_t*>(w + o_masks);
  uint32_t* boff = reinterpret_cast<uint32_t*>(w + o_boff);
  uint64_t* bst = reinterpret_cast<uint64_t*>(w + o_bst);
  uint32_t* stat = d_status ? d_status : reinterpret_cast<uint32_t*>(w + o_stat);
  const sks::ZeroSpans zs{{stat, reinterpret_cast<uint32_t*>(d_counts), ani ? static_cast<uint32_t*>(c->tdone.ptr) : nullptr},
                          {2, n_tiles * 4096, ani ? n_tiles : 0}};
  SKS_HIP(sks::join_layout_build(d_data, d_starts, d_sizes, n, log_b, elem_words, d_bounds, w + o_tmp, vals, masks,
                                 boff, bst, stat, c->join_check, c->stream, &zs, blocks_hint));
  const sks::JoinLayout L{vals, masks, boff, bst};
  sks::JoinAni A{d_ani, d_sizes_global, kmer_num_ones, static_cast<uint32_t*>(c->tdone.ptr)};
  if (ani && c->root_k == kmer_num_ones) {  // the context's table (sks_ctx_ani_table), if for this k
    A.root = static_cast<const double*>(c->root.ptr);
    A.root_size = c->root_size;
  }
  SKS_HIP(hipEventRecord(c->ev_begin, c->stream));
  // the layout's region log, as join_layout_build picks it: a tile list over
  // this one layout joins without cross-region windows when regions hold 64 buckets
  const int rg = (int)sks::join_layout_region_log(blocks_hint ? std::min(blocks_hint, nb) : nb, log_b);
  SKS_HIP(sks::join_launch(L, 0u - blk0, L, 0u - blk0, n_global, log_b, elem_words, true, 0, n_global, 0, n_tiles,
                           d_tiles, true, d_counts, c->join_check, c->stream, ani ? &A : nullptr, rg));
  SKS_HIP(hipEventRecord(c->ev_end, c->stream));
  return SKS_OK;
}

int sks_host_alloc(uint64_t bytes, int coherent, void** out) {
  if (!out) return sks::fail(SKS_E_ARG, "sks_host_alloc: null out");
  *out = nullptr;
  if (!bytes) return SKS_OK;
  void* p = nullptr;
  const unsigned flags = (coherent ? hipHostMallocCoherent : hipHostMallocNonCoherent) | hipHostMallocPortable |
                         hipHostMallocMapped;
  if (hipHostMalloc(&p, bytes, flags) != hipSuccess) {
    (void)hipGetLastError();
    return sks::fail(SKS_E_NOMEM, "sks_host_alloc: hipHostMalloc of " + std::to_string(bytes) + " bytes failed");
  }
  *out = p;
  return SKS_OK;
}

int sks_host_free(void* p) {
  if (p) SKS_HIP(hipHostFree(p));
  return SKS_OK;
}

int sks_ani_matrix(sks_ctx* c, const int32_t* d_counts, uint32_t n, int kmer_num_ones, double* d_cont,
                   double* d_ani) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ani_matrix: null ctx");
  if (kmer_num_ones <= 0) return sks::fail(SKS_E_ARG, "sks_ani_matrix: kmer_num_ones must be positive");
  if (n && (!d_counts || !d_ani)) return sks::fail(SKS_E_ARG, "sks_ani_matrix: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(sks::launch_ani_matrix(d_counts, n, kmer_num_ones, d_cont, d_ani, c->stream));
  return SKS_OK;
}

int sks_ani_rows(sks_ctx* c, const int32_t* d_counts, uint32_t n, uint32_t row_begin, uint32_t row_end,
                 int kmer_num_ones, double* d_cont, double* d_ani) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ani_rows: null ctx");
  if (kmer_num_ones <= 0) return sks::fail(SKS_E_ARG, "sks_ani_rows: kmer_num_ones must be positive");
  if (row_begin > row_end || row_end > n) return sks::fail(SKS_E_ARG, "sks_ani_rows: bad row range");
  if (row_end > row_begin && (!d_counts || !d_ani)) return sks::fail(SKS_E_ARG, "sks_ani_rows: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(sks::launch_ani_rows(d_counts, n, row_begin, row_end, kmer_num_ones, d_cont, d_ani, c->stream));
  return SKS_OK;
}

int sks_ani_tiles(sks_ctx* c, const int32_t* d_packed, const uint32_t* d_tiles, uint64_t n_tiles, uint32_t n,
                  const int32_t* d_sizes, int kmer_num_ones, double* d_ani) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_ani_tiles: null ctx");
  if (kmer_num_ones <= 0) return sks::fail(SKS_E_ARG, "sks_ani_tiles: kmer_num_ones must be positive");
  if (n_tiles && (!d_packed || !d_tiles || !d_sizes || !d_ani))
    return sks::fail(SKS_E_ARG, "sks_ani_tiles: null argument");
  DeviceGuard g(c->device);
  SKS_HIP(sks::launch_ani_tiles(d_packed, d_tiles, n_tiles, n, d_sizes, kmer_num_ones, d_ani, c->stream));
  return SKS_OK;
}

int sks_sketches_export(sks_ctx* c, const uint64_t* d_data, const uint64_t* d_starts, const uint32_t* d_sizes,
                        int elem_words, uint32_t n, uint64_t* d_dst, uint64_t stride, uint32_t* d_dst_sizes) {
  if (!c) return sks::fail(SKS_E_ARG, "sks_sketches_export: null ctx");
  if (elem_words != 1 && elem_words != 2) return sks::fail(SKS_E_ARG, "elem_words must be 1 or 2");
  if (n && (!d_starts || !d_sizes || !d_dst || !d_dst_sizes || !stride))
    return sks::fail(SKS_E_ARG, "sks_sketches_export: null argument or zero stride");
  DeviceGuard g(c->device);
  SKS_HIP(sks::launch_export(d_data, d_starts, d_sizes, n, elem_words, d_dst, stride, d_dst_sizes, c->stream));
  return SKS_OK;
}

int sks_sketch_set_export_csr(const sks_sketch_set* set, uint64_t* d_data, uint32_t* d_sizes) {
  if (!set) return sks::fail(SKS_E_ARG, "sks_sketch_set_export_csr: null set");
  DeviceGuard g(set->device);
  uint64_t total = 0;
  for (uint32_t v : set->sizes) total += v;
  if ((total && !d_data) || (set->n && !d_sizes))
    return sks::fail(SKS_E_ARG, "sks_sketch_set_export_csr: null argument");
  // the set's arrays are CSR in sketch order: one copy each
  if (total)
    SKS_HIP(hipMemcpy(d_data, set->d_data + set->starts[0] * set->elem_words,
                      total * set->elem_words * sizeof(uint64_t), hipMemcpyDeviceToDevice));
  if (set->n) SKS_HIP(hipMemcpy(d_sizes, set->d_sizes, set->n * sizeof(uint32_t), hipMemcpyDeviceToDevice));
  return SKS_OK;
}

// Device time of the last intersection call (after the stream has reached it).
int sks_ctx_last_intersect_ms(sks_ctx* c, float* ms) {
  if (!c || !ms) return sks::fail(SKS_E_ARG, "null argument");
  DeviceGuard g(c->device);
  SKS_HIP(hipEventSynchronize(c->ev_end));
  SKS_HIP(hipEventElapsedTime(ms, c->ev_begin, c->ev_end));
  return SKS_OK;
}

// ---- device FASTA ingress (ingress.hip) -----------------------------------------------------

int sks_fasta_parse_device(sks_ctx* c, const uint8_t* d_raw, uint64_t n_raw, uint8_t* d_stream,
                           uint64_t stream_cap, uint64_t* d_rec_end, uint64_t rec_cap,
                           uint64_t* stream_bytes, uint64_t* n_records) {
  if (!c || !stream_bytes || !n_records || (n_raw && !d_raw))
    return sks::fail(SKS_E_ARG, "sks_fasta_parse_device: null argument");
  DeviceGuard g(c->device);
  bool too_small = false;
  SKS_HIP(hipEventRecord(c->ev_i0, c->stream));
  SKS_HIP(sks::fasta_parse_device(d_raw, n_raw, d_stream, stream_cap, d_rec_end, rec_cap, c->ingress,
                                  c->tmp, c->stream, stream_bytes, n_records, &too_small));
  SKS_HIP(hipEventRecord(c->ev_i1, c->stream));
  if (too_small)
    return sks::fail(SKS_E_LENGTH, "sks_fasta_parse_device: stream_cap or rec_cap too small for " +
                                       std::to_string(*stream_bytes) + " bytes / " +
                                       std::to_string(*n_records) + " records");
  return SKS_OK;
}

int sks_ctx_last_ingress_ms(sks_ctx* c, float* ms) {
  if (!c || !ms) return sks::fail(SKS_E_ARG, "null argument");
  DeviceGuard g(c->device);
  SKS_HIP(hipEventSynchronize(c->ev_i1));
  SKS_HIP(hipEventElapsedTime(ms, c->ev_i0, c->ev_i1));
  return SKS_OK;
}

// ---- synthetic genomes ------------------------------------------------------------------------

int sks_synth_bases(sks_ctx* c, uint8_t* d_out, uint64_t n, uint64_t seed, uint64_t mut_seed,
                    double mut_rate, uint64_t pos_offset) {
  if (!c || (n && !d_out)) return sks::fail(SKS_E_ARG, "sks_synth_bases: null argument");
  uint64_t thr = 0;
  if (mut_rate > 0) {
    long double t = (long double)mut_rate * 18446744073709551616.0L;
    thr = t >= 18446744073709551615.0L ? ~0ull : (uint64_t)t;
  }
  DeviceGuard g(c->device);
  SKS_HIP(sks::launch_synth(d_out, n, seed, mut_seed, thr, pos_offset, c->stream));
  return SKS_OK;
}

}  // extern "C"
