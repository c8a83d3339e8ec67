// The reference-named C++ API (kmer.hpp, fasta_processing.hpp,
// ani_estimator.hpp) implemented on libsks.so's C ABI.  Sketching and
// intersection go to the GPU; only ingress bookkeeping, masks, hashing of
// single k-mers and the final double arithmetic run on the host — as in the
// reference, where those are host code too.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <functional>
#include <iostream>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>

#include "ani_estimator.hpp"
#include "fasta_processing.hpp"
#include "kmer.hpp"
#include "sks.h"
#include "sks_api_internal.hpp"
#include "sks_hash.hpp"
#include "facade_internal.hpp"

namespace sks {
namespace {

std::mutex g_mu;
int g_device = 0;
bool g_device_set = false;
sks_ctx* g_ctx = nullptr;
bool g_exit_on_io = true;
int g_flavour = SKS_HASH_BOOST_MIX;

}  // namespace

[[noreturn]] void raise(int rc) {
  throw std::runtime_error(std::string("libsks: ") + sks_last_error() + " (status " +
                           std::to_string(rc) + ")");
}

void check(int rc) {
  if (rc != SKS_OK) raise(rc);
}

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

sks_ctx* ctx() {
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_ctx) check(sks_ctx_create(g_device, nullptr, &g_ctx));
  return g_ctx;
}

DevMem::DevMem(size_t n, int dev) : device(dev < 0 ? g_device : dev), bytes(n) {
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipMalloc(&p, n ? n : 1), "hipMalloc");
}

DevMem::~DevMem() {
  if (p) {
    (void)hipSetDevice(device);
    (void)hipFree(p);
  }
}

sks_fasta* open_fasta(const char* path) {
  sks_fasta* f = nullptr;
  int rc = sks_fasta_open(path, &f);
  if (rc == SKS_E_IO && g_exit_on_io) {
    // fasta_processing.cpp:86-90
    std::cerr << "Unable to open " << path << ". \n Exiting..." << std::endl;
    exit(1);
  }
  check(rc);
  return f;
}

struct FastaHandle {
  sks_fasta* f;
  explicit FastaHandle(const char* path) : f(open_fasta(path)) {}
  ~FastaHandle() { sks_fasta_close(f); }
};

// Sketch a device buffer of consecutive segments (off[i], off[i+1]) in one build.
std::vector<kmer_set> sketch_device(sks_ctx* c, const uint8_t* d_seq, const std::vector<uint64_t>& off,
                                    const kmer_bitset& mask, int w, const sketch_policy& pol) {
  const size_t n_seg = off.size() - 1;
  sks_policy p{pol.kind, pol.flavour, pol.param, pol.nonce};
  uint64_t m[2] = {mask.lo(), mask.hi()};
  sks_sketch_set* set = nullptr;
  check(sks_sketch_build(c, d_seq, off.back(), off.data(), (uint32_t)n_seg, w, m, &p, &set));
  const int ew = sks_sketch_set_elem_words(set);
  std::vector<uint32_t> sizes(n_seg);
  sks_sketch_set_sizes(set, sizes.data());
  std::vector<kmer_set> out(n_seg);
  std::vector<uint64_t> buf;
  for (size_t i = 0; i < n_seg; ++i) {
    buf.resize((size_t)sizes[i] * ew);
    int rc = sks_sketch_set_copy(set, (uint32_t)i, buf.data());
    if (rc != SKS_OK) {
      sks_sketch_set_free(set);
      raise(rc);
    }
    kmer_set& ks = out[i];
    ks.window_length = w;
    ks.mask = mask;
    ks.has_mask = true;
    ks.elements.resize(sizes[i]);
    for (uint32_t e = 0; e < sizes[i]; ++e)
      ks.elements[e] = ew == 1 ? kmer_bitset(buf[e], 0) : kmer_bitset(buf[2 * e], buf[2 * e + 1]);
  }
  sks_sketch_set_free(set);
  return out;
}

// Upload record streams (already parsed) as consecutive segments and sketch them.
std::vector<kmer_set> sketch_streams(const std::vector<std::vector<uint8_t>>& streams,
                                     const kmer_bitset& mask, int w, const sketch_policy& pol) {
  std::vector<uint64_t> off(1, 0);
  for (auto& s : streams) off.push_back(off.back() + s.size());
  std::vector<uint8_t> all;
  all.reserve(off.back());
  for (auto& s : streams) all.insert(all.end(), s.begin(), s.end());
  DevMem d(all.size());
  check_hip(hipMemcpy(d.p, all.data(), all.size(), hipMemcpyHostToDevice), "hipMemcpy H2D");
  return sketch_device(ctx(), d.as<uint8_t>(), off, mask, w, pol);
}

// Raw FASTA files: the host only reads bytes; strings_from_fasta runs on the
// device (sks_fasta_parse_device) straight into the segment layout.
std::vector<kmer_set> sketch_raw_files(sks_ctx* c, int device,
                                       const std::vector<const std::vector<uint8_t>*>& raws,
                                       const kmer_bitset& mask, int w, const sketch_policy& pol) {
  std::vector<uint64_t> in_off(1, 0);
  for (auto* r : raws) in_off.push_back(in_off.back() + r->size());
  DevMem d_raw(in_off.back(), device);
  for (size_t i = 0; i < raws.size(); ++i)
    if (!raws[i]->empty())
      check_hip(hipMemcpy(d_raw.as<uint8_t>() + in_off[i], raws[i]->data(), raws[i]->size(),
                          hipMemcpyHostToDevice), "hipMemcpy H2D");
  DevMem d_stream(in_off.back() + raws.size(), device);  // a stream is at most raw + 1 bytes
  std::vector<uint64_t> off(1, 0);
  for (size_t i = 0; i < raws.size(); ++i) {
    uint64_t nb = 0, nr = 0;
    check(sks_fasta_parse_device(c, d_raw.as<uint8_t>() + in_off[i], raws[i]->size(),
                                 d_stream.as<uint8_t>() + off.back(), raws[i]->size() + 1, nullptr, 0,
                                 &nb, &nr));
    off.push_back(off.back() + nb);
  }
  return sketch_device(c, d_stream.as<uint8_t>(), off, mask, w, pol);
}

std::vector<kmer_set> sketch_raw_files(const std::vector<std::vector<uint8_t>>& raws,
                                       const kmer_bitset& mask, int w, const sketch_policy& pol) {
  std::vector<const std::vector<uint8_t>*> r;
  for (auto& x : raws) r.push_back(&x);
  return sketch_raw_files(ctx(), g_device, r, mask, w, pol);
}

// ---- device pool of the parallel_* entry points ---------------------------------------------
namespace {
std::vector<int> g_devices;  // set_devices; empty = default
struct PoolCtx {
  int device;
  sks_ctx* ctx;
};
std::vector<PoolCtx> g_pool;  // one context per list entry (a repeated device gets several)

std::vector<int> default_devices() {
  if (const char* e = getenv("SKS_FACADE_DEVICES")) {
    std::vector<int> d;
    for (const char* q = e; *q;) {
      char* end = nullptr;
      const long v = strtol(q, &end, 10);
      if (end == q) break;
      d.push_back((int)v);
      q = *end == ',' ? end + 1 : end;
    }
    if (!d.empty()) return d;
  }
  if (g_device_set) return {g_device};
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return {g_device};
  std::vector<int> d(n);
  std::iota(d.begin(), d.end(), 0);
  return d;
}
}  // namespace

std::vector<int> pool_devices() {
  std::lock_guard<std::mutex> lock(g_mu);
  return g_devices.empty() ? default_devices() : g_devices;
}

// Context of pool entry i (created on first use; entries persist for the process).
sks_ctx* pool_ctx(size_t i, int device) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_pool.size() <= i) g_pool.resize(i + 1, PoolCtx{-1, nullptr});
  PoolCtx& p = g_pool[i];
  if (p.ctx && p.device != device) {
    sks_ctx_destroy(p.ctx);
    p.ctx = nullptr;
  }
  if (!p.ctx) {
    check(sks_ctx_create(device, nullptr, &p.ctx));
    p.device = device;
  }
  return p.ctx;
}

// Runs job(k, device, ctx) for k in [0, n_parts) on the pool, one host thread
// per part; the first exception (in part order) is rethrown.
void on_pool(size_t n_parts, const std::vector<int>& devs,
             const std::function<void(size_t, int, sks_ctx*)>& job) {
  std::vector<std::exception_ptr> err(n_parts);
  std::vector<sks_ctx*> cs(n_parts);
  for (size_t k = 0; k < n_parts; ++k) cs[k] = pool_ctx(k, devs[k]);
  std::vector<std::thread> ts;
  for (size_t k = 0; k < n_parts; ++k)
    ts.emplace_back([&, k]() {
      try {
        check_hip(hipSetDevice(devs[k]), "hipSetDevice");
        job(k, devs[k], cs[k]);
      } catch (...) {
        err[k] = std::current_exception();
      }
    });
  for (auto& t : ts) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

// Whole-file read; false if the file cannot be opened or read.
bool read_raw(const char* path, std::vector<uint8_t>& buf) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  buf.clear();
  uint8_t tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
  bool ok = !ferror(f);
  fclose(f);
  return ok;
}

// The reference's missing-file behaviour (fasta_processing.cpp:86-90).
void report_unreadable(const char* path) {
  FastaHandle f(path);  // exits (or throws) like the reference
}


std::vector<std::vector<uint8_t>> read_files(int num_files, char* filenames[]) {
  const int n = num_files > 0 ? num_files : 0;
  std::vector<std::vector<uint8_t>> raws(n);
  // open serially first so that the reference's exit(1) / error order holds
  for (int i = 0; i < n; ++i) {
    FILE* fp = fopen(filenames[i], "rb");
    if (!fp) report_unreadable(filenames[i]);
    else fclose(fp);
  }
  std::vector<int> bad(n, 0);
  const int workers = std::max(1, std::min<int>(n, (int)std::thread::hardware_concurrency()));
  std::vector<std::thread> ts;
  std::atomic<int> next{0};
  for (int t = 0; t < workers; ++t)
    ts.emplace_back([&]() {
      for (int i; (i = next.fetch_add(1)) < n;)
        if (!read_raw(filenames[i], raws[i])) bad[i] = 1;
    });
  for (auto& t : ts) t.join();
  for (int i = 0; i < n; ++i)
    if (bad[i]) report_unreadable(filenames[i]);
  return raws;
}

namespace {

// Devices of the pair count in progress: empty = the facade's own context
// (compute_pairwise_...), else the pool (parallel_compute_pairwise_...).
thread_local std::vector<int> g_pair_devices;
std::mutex g_pair_stats_mu;
pair_flow_stats g_pair_stats{};
struct PairDevices {  // scope of a parallel_ pair count (one device keeps the facade's context)
  std::vector<int> saved;
  explicit PairDevices(std::vector<int> d) : saved(std::move(g_pair_devices)) {
    g_pair_devices = d.size() >= 2 ? std::move(d) : std::vector<int>{};
  }
  ~PairDevices() { g_pair_devices = std::move(saved); }
};

// Pair counts on the GPU for sets sharing a mask; pairs with different masks
// have no common k-mer (identity includes the mask, kmer.hpp:82-85).
std::vector<int> pair_counts_single_mask(const std::vector<const kmer_set*>& a,
                                         const std::vector<const kmer_set*>& b);

// Sets holding k-mers under several masks: identity is (masked_bits, mask)
// (kmer.hpp:82-85), so |A ∩ B| = Σ over masks m held by both of |A_m ∩ B_m|.
// Each (set, mask) part becomes one sketch; the parts sharing a mask are counted
// on the GPU (sks_intersect_pairs) and summed per pair.
std::vector<int> pair_counts_mixed(const std::vector<const kmer_set*>& a,
                                   const std::vector<const kmer_set*>& b) {
  std::vector<kmer_set> parts;  // single-mask views of every (set, mask) part
  std::vector<const kmer_set*> pa, pb;
  std::vector<size_t> owner;
  std::unordered_map<const void*, size_t> part_of;  // &elements -> index in parts
  auto part = [&](const kmer_set* s, size_t g) {
    const std::vector<kmer_bitset>* e = g == 0 ? &s->elements : &s->other_masks[g - 1].elements;
    auto it = part_of.find(e);
    if (it != part_of.end()) return it->second;
    kmer_set p;
    p.has_mask = true;
    p.mask = g == 0 ? s->mask : s->other_masks[g - 1].mask;
    p.window_length = g == 0 ? s->window_length : s->other_masks[g - 1].window_length;
    p.elements = *e;
    parts.push_back(std::move(p));
    part_of.emplace(e, parts.size() - 1);
    return parts.size() - 1;
  };
  std::vector<std::pair<size_t, size_t>> sub;
  for (size_t i = 0; i < a.size(); ++i) {
    for (size_t ga = 0; ga <= a[i]->other_masks.size(); ++ga) {
      const kmer_bitset& m = ga == 0 ? a[i]->mask : a[i]->other_masks[ga - 1].mask;
      if (ga == 0 && !a[i]->has_mask) continue;
      for (size_t gb = 0; gb <= b[i]->other_masks.size(); ++gb) {
        if (gb == 0 && !b[i]->has_mask) continue;
        const kmer_bitset& mb = gb == 0 ? b[i]->mask : b[i]->other_masks[gb - 1].mask;
        if (!(m == mb)) continue;
        sub.emplace_back(part(a[i], ga), part(b[i], gb));
        owner.push_back(i);
      }
    }
  }
  std::vector<int> out(a.size(), 0);
  if (sub.empty()) return out;
  for (auto& [x, y] : sub) {  // parts is final now
    pa.push_back(&parts[x]);
    pb.push_back(&parts[y]);
  }
  const std::vector<int> c = pair_counts_single_mask(pa, pb);
  for (size_t k = 0; k < sub.size(); ++k) out[owner[k]] += c[k];
  return out;
}

std::vector<int> pair_counts(const std::vector<const kmer_set*>& a,
                             const std::vector<const kmer_set*>& b) {
  for (size_t i = 0; i < a.size(); ++i)
    if (!a[i]->other_masks.empty() || !b[i]->other_masks.empty()) return pair_counts_mixed(a, b);
  return pair_counts_single_mask(a, b);
}

std::vector<int> pair_counts_single_mask(const std::vector<const kmer_set*>& a,
                                         const std::vector<const kmer_set*>& b) {
  std::unordered_map<const kmer_set*, int32_t> index;
  std::vector<const kmer_set*> uniq;
  auto id = [&](const kmer_set* s) {
    auto it = index.find(s);
    if (it != index.end()) return it->second;
    int32_t k = (int32_t)uniq.size();
    index.emplace(s, k);
    uniq.push_back(s);
    return k;
  };
  std::vector<int32_t> ia(a.size()), ib(b.size());
  for (size_t i = 0; i < a.size(); ++i) {
    ia[i] = id(a[i]);
    ib[i] = id(b[i]);
  }
  int ew = 1;
  for (auto* s : uniq)
    for (auto& e : s->elements)
      if (e.hi()) ew = 2;
  std::vector<uint64_t> starts(uniq.size()), words;
  std::vector<uint32_t> sizes(uniq.size());
  uint64_t total = 0;
  for (size_t i = 0; i < uniq.size(); ++i) {
    starts[i] = total;
    sizes[i] = (uint32_t)uniq[i]->elements.size();
    total += sizes[i];
    for (auto& e : uniq[i]->elements) {
      words.push_back(e.lo());
      if (ew == 2) words.push_back(e.hi());
    }
  }
  std::vector<int> out(a.size(), 0);
  if (a.empty()) return out;
  std::vector<int32_t> res(a.size());
  const uint64_t n = uniq.size();
  // Pair lists that cover a large part of the n x n matrix — the reference's
  // main flow intersects generate_all_pairs_from_vector's list
  // (kmer-sketching.cpp:195-200) — are counted as the whole symmetric matrix by
  // the join (one layout of all n sketches, its 64 x 64 upper-triangle tiles)
  // and gathered; sparse lists go through one wavefront per pair
  // (sks_intersect_pairs).
  const bool dense = n >= 64 && n <= 16384 && a.size() * 4 >= n * n;
  // parallel_* callers spread the work over the device pool (kmer_set.cpp:
  // 167-184's cilk_for over pairs): each pool entry counts a contiguous share
  // of the tiles (dense) or of the pair list
  const std::vector<int> devs = g_pair_devices.empty() ? std::vector<int>{g_device} : g_pair_devices;
  const uint64_t T = dense ? sks_intersect_sym_tiles((uint32_t)n) : 0;
  const uint64_t units = dense ? T : a.size();
  const size_t parts = (size_t)std::max<uint64_t>(1, std::min<uint64_t>(devs.size(), units));
  // The sketches cross PCIe once, to the first pool device; every other device
  // of the pool gets a device-to-device copy (xGMI peer copy between GPUs; a
  // pool entry repeating a device shares its copy)
  struct Resident {
    int device;
    std::unique_ptr<DevMem> words, starts, sizes;
  };
  std::vector<Resident> res_dev;
  auto resident_on = [&](int device) -> const Resident& {
    for (auto& r : res_dev)
      if (r.device == device) return r;
    Resident r{device, std::unique_ptr<DevMem>(new DevMem(words.size() * 8, device)),
               std::unique_ptr<DevMem>(new DevMem(starts.size() * 8, device)),
               std::unique_ptr<DevMem>(new DevMem(sizes.size() * 4, device))};
    const uint64_t bytes = words.size() * 8 + starts.size() * 8 + sizes.size() * 4;
    if (res_dev.empty()) {
      check_hip(hipMemcpy(r.words->p, words.data(), words.size() * 8, hipMemcpyHostToDevice), "H2D");
      check_hip(hipMemcpy(r.starts->p, starts.data(), starts.size() * 8, hipMemcpyHostToDevice), "H2D");
      check_hip(hipMemcpy(r.sizes->p, sizes.data(), sizes.size() * 4, hipMemcpyHostToDevice), "H2D");
      std::lock_guard<std::mutex> lock(g_pair_stats_mu);
      g_pair_stats.h2d_bytes += bytes;
    } else {
      const Resident& src = res_dev.front();
      check_hip(hipMemcpyPeer(r.words->p, device, src.words->p, src.device, words.size() * 8), "D2D");
      check_hip(hipMemcpyPeer(r.starts->p, device, src.starts->p, src.device, starts.size() * 8), "D2D");
      check_hip(hipMemcpyPeer(r.sizes->p, device, src.sizes->p, src.device, sizes.size() * 4), "D2D");
      std::lock_guard<std::mutex> lock(g_pair_stats_mu);
      g_pair_stats.d2d_bytes += bytes;
    }
    res_dev.push_back(std::move(r));
    return res_dev.back();
  };
  std::vector<const Resident*> on(parts);
  for (size_t k = 0; k < parts; ++k) on[k] = &resident_on(devs[k]);  // before the pool threads start
  std::vector<int32_t> mat(dense ? n * n : 0, 0);
  std::mutex mat_mu;
  auto job = [&](size_t k, int device, sks_ctx* c) {
    const uint64_t u0 = units * k / parts, u1 = units * (k + 1) / parts;
    if (u1 <= u0) return;
    const Resident& R = *on[k];
    const uint64_t* dw = R.words->as<uint64_t>();
    const uint64_t* ds = R.starts->as<uint64_t>();
    const uint32_t* dz = R.sizes->as<uint32_t>();
    if (dense) {
      // the layout of all n sketches, then this part's tiles [u0, u1), packed
      // (16 KB a tile): only its own tiles come back
      uint32_t max_size = 1;
      for (uint32_t v : sizes) max_size = std::max(max_size, v);
      const uint32_t log_b = sks_join_layout_log_b(max_size);
      const uint64_t nb = (n + 63) / 64, tot = std::max<uint64_t>(total, 1);
      DevMem vals(tot * 8 * ew, device), masks(tot * 8, device),
          boff(nb * sks_join_layout_boff_words(log_b) * 4, device), bst((nb + 1) * 8, device);
      uint32_t stat = 0;
      check(sks_join_layout_build(c, dw, ds, dz, ew, (uint32_t)n, tot, log_b, nullptr, vals.as<uint64_t>(),
                                  masks.as<uint64_t>(), boff.as<uint32_t>(), bst.as<uint64_t>(), &stat));
      const uint64_t nt = u1 - u0;
      DevMem tiles_out(nt * 4096 * 4, device);
      check_hip(hipMemset(tiles_out.p, 0, nt * 4096 * 4), "hipMemset");  // the join adds into its tiles
      check(sks_intersect_layout_tiles(c, (uint32_t)n, log_b, ew, vals.as<uint64_t>(), masks.as<uint64_t>(),
                                       boff.as<uint32_t>(), bst.as<uint64_t>(), 0, nullptr, u0, u1, 1,
                                       tiles_out.as<int32_t>()));
      check(sks_ctx_synchronize(c));
      std::vector<int32_t> h(nt * 4096);
      check_hip(hipMemcpy(h.data(), tiles_out.p, nt * 4096 * 4, hipMemcpyDeviceToHost), "D2H");
      std::lock_guard<std::mutex> lock(mat_mu);
      g_pair_stats.d2h_bytes += nt * 4096 * 4;
      for (uint64_t t = u0; t < u1; ++t) {  // upper-triangle tile t, row-major (I <= J)
        uint64_t I = 0, r = t;
        while (r >= nb - I) {
          r -= nb - I;
          ++I;
        }
        const uint64_t J = I + r;
        const int32_t* tl = h.data() + (t - u0) * 4096;
        for (uint64_t y = 0; y < 64 && I * 64 + y < n; ++y)
          for (uint64_t x = 0; x < 64 && J * 64 + x < n; ++x) {
            const int32_t v = tl[y * 64 + x];
            mat[(I * 64 + y) * n + J * 64 + x] = v;
            mat[(J * 64 + x) * n + I * 64 + y] = v;
          }
      }
    } else {
      const uint64_t m = u1 - u0;
      DevMem d_a(m * 4, device), d_b(m * 4, device), d_out(m * 4, device);
      check_hip(hipMemcpy(d_a.p, ia.data() + u0, m * 4, hipMemcpyHostToDevice), "H2D");
      check_hip(hipMemcpy(d_b.p, ib.data() + u0, m * 4, hipMemcpyHostToDevice), "H2D");
      check(sks_intersect_pairs(c, dw, ds, dz, ew, d_a.as<int32_t>(), d_b.as<int32_t>(), m, d_out.as<int32_t>()));
      check(sks_ctx_synchronize(c));
      check_hip(hipMemcpy(res.data() + u0, d_out.p, m * 4, hipMemcpyDeviceToHost), "D2H");
      std::lock_guard<std::mutex> lock(g_pair_stats_mu);
      g_pair_stats.h2d_bytes += 2 * m * 4;
      g_pair_stats.d2h_bytes += m * 4;
    }
  };
  if (g_pair_devices.empty()) job(0, g_device, ctx());
  else on_pool(parts, devs, job);
  {
    std::lock_guard<std::mutex> lock(g_pair_stats_mu);
    ++g_pair_stats.calls;
    g_pair_stats.devices += parts;
  }
  if (dense)
    for (size_t i = 0; i < a.size(); ++i) res[i] = mat[(uint64_t)ia[i] * n + ib[i]];
  for (size_t i = 0; i < a.size(); ++i) {
    const bool same = a[i]->mask == b[i]->mask || a[i]->elements.empty() || b[i]->elements.empty();
    out[i] = same ? res[i] : 0;
  }
  return out;
}

}  // namespace

void set_device(int device) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_ctx && device != g_device) {
    sks_ctx_destroy(g_ctx);
    g_ctx = nullptr;
  }
  g_device = device;
  g_device_set = true;
}

void set_devices(const std::vector<int>& devices) {
  std::lock_guard<std::mutex> lock(g_mu);
  g_devices = devices;
}

std::vector<int> parallel_devices() { return pool_devices(); }

void set_exit_on_io_error(bool exit_on_error) { g_exit_on_io = exit_on_error; }
void set_hash_flavour(int flavour) { g_flavour = flavour; }
int hash_flavour() { return g_flavour; }
uint64_t bitset_hash(const kmer_bitset& b) { return hash_bitset128_rt(b.lo(), b.hi(), g_flavour); }

}  // namespace sks

// ---- masks ---------------------------------------------------------------------------------------
void initialise_contiguous_kmer_array() {}  // tables are not needed (kept for source compatibility)
void initialise_reversing_kmer_array() {}

kmer_bitset contiguous_kmer(const int kmer_length) {
  uint64_t m[2];
  if (kmer_length > MAX_KMER_LENGTH)
    throw std::runtime_error("Given k-mer length exceeds maximum k-mer length");
  sks::check(sks_mask_contiguous(kmer_length, m));
  return kmer_bitset(m[0], m[1]);
}

// kmer_bitset.cpp:88-99: reverses the order of the 64 two-bit groups.
kmer_bitset reverse_kmer_bitset(const kmer_bitset& kbs) {
  kmer_bitset r;
  for (int g = 0; g < MAX_KMER_LENGTH; ++g) {
    int src = 2 * g, dst = 2 * (MAX_KMER_LENGTH - 1 - g);
    r.set(dst, kbs.test(src));
    r.set(dst + 1, kbs.test(src + 1));
  }
  return r;
}

kmer_bitset generate_random_spaced_seed_mask(const int window_size, const int kmer_size,
                                             size_t random_seed) {
  uint64_t m[2];
  int rc = sks_mask_generate(window_size, kmer_size, random_seed, m);
  if (rc != SKS_OK) throw std::invalid_argument(sks_last_error());
  return kmer_bitset(m[0], m[1]);
}

// kmers.cpp:16-35
kmer reverse_complement(kmer k) {
  kmer_bitset rc = reverse_kmer_bitset(k.kmer_bits).flip() >>
                   ((MAX_KMER_LENGTH - k.window_length) * NUCLEOTIDE_BIT_SIZE);
  return {k.window_length, rc, k.mask, rc & k.mask};
}

kmer canonical_kmer(kmer k) {
  kmer rc = reverse_complement(k);
  return (k.masked_bits < rc.masked_bits) ? k : rc;
}

// kmer.hpp:135-149: H(masked_bits) ^ (H(mask) ^ hash<int>(w) ^ nonce).  The
// second part depends on the mask, window and nonce only; a predicate calls
// this once per window with the same three, so the last one is kept per thread.
size_t frac_min_hash::operator()(const kmer& k) const {
  struct Memo {
    uint64_t mlo = 0, mhi = 0, value = 0;
    int w = -1, nonce = 0, flavour = -1;
  };
  thread_local Memo memo;
  const uint64_t mlo = k.mask.lo(), mhi = k.mask.hi();
  if (memo.w != k.window_length || memo.mlo != mlo || memo.mhi != mhi || memo.nonce != nonce ||
      memo.flavour != flavour) {
    memo.value = sks::fmh_const(mlo, mhi, k.window_length, nonce, flavour);
    memo.mlo = mlo;
    memo.mhi = mhi;
    memo.w = k.window_length;
    memo.nonce = nonce;
    memo.flavour = flavour;
  }
  return sks::hash_bitset128_rt(k.masked_bits.lo(), k.masked_bits.hi(), flavour) ^ memo.value;
}

// ---- kmer_set -------------------------------------------------------------------------------------
namespace {
// insert sorted masked bits into a sorted unique array
void merge_into(std::vector<kmer_bitset>& dst, std::vector<kmer_bitset>& add) {
  std::sort(add.begin(), add.end());
  std::vector<kmer_bitset> merged;
  merged.reserve(dst.size() + add.size());
  std::merge(dst.begin(), dst.end(), add.begin(), add.end(), std::back_inserter(merged));
  merged.erase(std::unique(merged.begin(), merged.end()), merged.end());
  dst.swap(merged);
}
}  // namespace

void kmer_set::insert_kmers(const std::vector<kmer>& kmers) {
  if (kmers.empty()) return;
  std::vector<kmer_bitset> add;
  std::vector<std::vector<kmer_bitset>> add_other(other_masks.size());
  add.reserve(kmers.size());
  for (const kmer& k : kmers) {
    if (!has_mask) {
      mask = k.mask;
      window_length = k.window_length;
      has_mask = true;
    }
    if (k.mask == mask) {
      add.push_back(k.masked_bits);
      continue;
    }
    size_t g = 0;
    while (g < other_masks.size() && !(other_masks[g].mask == k.mask)) ++g;
    if (g == other_masks.size()) {
      other_masks.push_back(mask_group{k.window_length, k.mask, {}});
      add_other.emplace_back();
    }
    add_other[g].push_back(k.masked_bits);
  }
  merge_into(elements, add);
  for (size_t g = 0; g < other_masks.size(); ++g)
    if (!add_other[g].empty()) merge_into(other_masks[g].elements, add_other[g]);
}

int kmer_set::kmer_set_size() const {
  size_t n = elements.size();
  for (const auto& g : other_masks) n += g.elements.size();
  return (int)n;
}

const std::vector<kmer_bitset>* kmer_set::elements_for(const kmer_bitset& m) const {
  if (has_mask && m == mask) return &elements;
  for (const auto& g : other_masks)
    if (g.mask == m) return &g.elements;
  return nullptr;
}

bool kmer_set::contains(const kmer& k) const {
  const std::vector<kmer_bitset>* e = elements_for(k.mask);
  return e && std::binary_search(e->begin(), e->end(), k.masked_bits);
}

// ---- kmer_hashes view --------------------------------------------------------------------------------
namespace {
size_t n_groups(const kmer_set* s) { return 1 + s->other_masks.size(); }
const std::vector<kmer_bitset>& group_elems(const kmer_set* s, size_t g) {
  return g == 0 ? s->elements : s->other_masks[g - 1].elements;
}
kmer group_kmer(const kmer_set* s, size_t g, size_t e) {
  const kmer_bitset& b = group_elems(s, g)[e];
  if (g == 0) return kmer{s->window_length, b, s->mask, b};
  const auto& grp = s->other_masks[g - 1];
  return kmer{grp.window_length, b, grp.mask, b};
}
}  // namespace

void kmer_hash_view::const_iterator::settle() {
  while (g_ < n_groups(s_) && e_ >= group_elems(s_, g_).size()) {
    ++g_;
    e_ = 0;
  }
  if (g_ < n_groups(s_)) cur_.emplace(group_kmer(s_, g_, e_), 1);
  else cur_.reset();
}

std::size_t kmer_hash_view::size() const { return (std::size_t)s_->kmer_set_size(); }
std::size_t kmer_hash_view::count(const kmer& k) const { return s_->contains(k) ? 1 : 0; }
int kmer_hash_view::at(const kmer& k) const {
  if (!s_->contains(k)) throw std::out_of_range("kmer_set::kmer_hashes::at: k-mer not in the set");
  return 1;
}
kmer_hash_view::const_iterator kmer_hash_view::begin() const { return const_iterator(s_, 0, 0); }
kmer_hash_view::const_iterator kmer_hash_view::end() const { return const_iterator(s_, n_groups(s_), 0); }
kmer_hash_view::const_iterator kmer_hash_view::find(const kmer& k) const {
  for (size_t g = 0; g < n_groups(s_); ++g) {
    const bool same = g == 0 ? (s_->has_mask && s_->mask == k.mask) : s_->other_masks[g - 1].mask == k.mask;
    if (!same) continue;
    const auto& e = group_elems(s_, g);
    auto it = std::lower_bound(e.begin(), e.end(), k.masked_bits);
    if (it != e.end() && *it == k.masked_bits) return const_iterator(s_, g, (size_t)(it - e.begin()));
  }
  return end();
}

int kmer_set_intersection(const kmer_set& ks1, const kmer_set& ks2) {
  return sks::pair_counts({&ks1}, {&ks2})[0];
}

// ---- sketch builders ---------------------------------------------------------------------------------
kmer_set kmer_set_from_fasta_file(const char fasta_filename[], const kmer_bitset& mask,
                                  const int window_length, const sketch_policy& policy) {
  char* names[1] = {const_cast<char*>(fasta_filename)};
  return kmer_sets_from_fasta_files(1, names, mask, window_length, policy)[0];
}

std::vector<kmer_set> kmer_sets_from_fasta_files(const int num_files, char* fasta_filenames[],
                                                 const kmer_bitset& mask, const int window_length,
                                                 const sketch_policy& policy) {
  std::vector<std::vector<uint8_t>> raws(num_files > 0 ? num_files : 0);
  for (int i = 0; i < num_files; ++i)
    if (!sks::read_raw(fasta_filenames[i], raws[i])) sks::report_unreadable(fasta_filenames[i]);
  return sks::sketch_raw_files(raws, mask, window_length, policy);
}

std::vector<kmer_set> parallel_kmer_sets_from_fasta_files(const int num_files,
                                                          char* fasta_filenames[],
                                                          const kmer_bitset& mask,
                                                          const int window_length,
                                                          const sketch_policy& policy) {
  // the reference's cilk_for over files (kmer_set.cpp:112-133) on the node's
  // GPUs: the files are cut into one contiguous range per device of about equal
  // bytes, each range parsed and sketched in one batched build on its device
  const std::vector<std::vector<uint8_t>> raws = sks::read_files(num_files, fasta_filenames);
  const std::vector<int> devs = sks::pool_devices();
  const size_t n = raws.size(), parts = std::min(devs.size(), n);
  if (parts < 2) return sks::sketch_raw_files(raws, mask, window_length, policy);
  uint64_t total = 0;
  for (auto& r : raws) total += r.size() + 1;
  std::vector<size_t> cut(1, 0);  // part k holds files [cut[k], cut[k + 1])
  uint64_t acc = 0;
  for (size_t i = 0; i < n && cut.size() < parts; ++i) {
    acc += raws[i].size() + 1;
    // close part k once it reaches its share, leaving a file for every later part
    if (acc * parts >= total * cut.size() && n - (i + 1) >= parts - cut.size()) cut.push_back(i + 1);
  }
  while (cut.size() < parts) cut.push_back(cut.back());
  cut.push_back(n);
  std::vector<std::vector<kmer_set>> part_out(parts);
  sks::on_pool(parts, devs, [&](size_t k, int device, sks_ctx* c) {
    std::vector<const std::vector<uint8_t>*> mine;
    for (size_t i = cut[k]; i < cut[k + 1]; ++i) mine.push_back(&raws[i]);
    if (!mine.empty()) part_out[k] = sks::sketch_raw_files(c, device, mine, mask, window_length, policy);
  });
  std::vector<kmer_set> out;
  out.reserve(n);
  for (auto& po : part_out)
    for (auto& ks : po) out.push_back(std::move(ks));
  return out;
}

namespace {
// acgt_strings -> record stream; codes act through their low two bits like the
// reference's update_kmer_window (kmer_sliding.cpp:26-47).
std::vector<uint8_t> runs_stream(const std::vector<std::vector<uint8_t>>& nucleotide_strings) {
  static const char kAcgt[4] = {'A', 'C', 'G', 'T'};
  std::vector<uint8_t> s;
  for (const auto& run : nucleotide_strings) {
    for (uint8_t b : run) s.push_back((uint8_t)kAcgt[b & 3]);
    s.push_back('\n');
  }
  return s;
}
}  // namespace

kmer_set nucleotide_string_list_to_kmer_set(const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                            const kmer_bitset& mask, const int window_length,
                                            const sketch_policy& policy) {
  return sks::sketch_streams({runs_stream(nucleotide_strings)}, mask, window_length, policy)[0];
}

void nucleotide_string_list_to_kmers_by_reference(std::vector<kmer>& kmer_list,
                                                  const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketch_policy& sketching_cond) {
  if (sketching_cond.kind != SKS_FRAC_MOD)
    throw std::invalid_argument("nucleotide_string_list_to_kmers: needs a per-k-mer (FracMinHash) condition");
  const std::vector<uint8_t> s = runs_stream(nucleotide_strings);
  if (s.empty()) return;
  sks::DevMem d(s.size());
  sks::check_hip(hipMemcpy(d.p, s.data(), s.size(), hipMemcpyHostToDevice), "hipMemcpy H2D");
  sks_policy p{sketching_cond.kind, sketching_cond.flavour, sketching_cond.param, sketching_cond.nonce};
  const uint64_t m[2] = {mask.lo(), mask.hi()};
  const uint64_t seg[2] = {0, s.size()};
  sks_kmer_list* kl = nullptr;
  sks::check(sks_kmer_list_build(sks::ctx(), d.as<uint8_t>(), s.size(), seg, 1, window_length, m, &p, &kl));
  const uint64_t n = sks_kmer_list_total(kl);
  std::vector<uint64_t> bits(4 * n);
  const int rc = sks_kmer_list_copy(kl, nullptr, bits.data());
  sks_kmer_list_free(kl);
  sks::check(rc);
  kmer_list.reserve(kmer_list.size() + n);
  for (uint64_t i = 0; i < n; ++i)
    kmer_list.push_back(kmer{window_length, kmer_bitset(bits[4 * i], bits[4 * i + 1]), mask,
                             kmer_bitset(bits[4 * i + 2], bits[4 * i + 3])});
}

std::vector<kmer> nucleotide_string_list_to_kmers(const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketch_policy& sketching_cond) {
  std::vector<kmer> out;
  nucleotide_string_list_to_kmers_by_reference(out, nucleotide_strings, mask, window_length,
                                               sketching_cond);
  return out;
}

// ---- the std::function plug-in point (kmer.hpp:93-103, :195-212) ----------------------------------------
namespace sks {
namespace {

// A worker of the host-predicate flow: its own context on its own HIP stream,
// and double buffers (device and pinned host) for one piece of record stream
// in and its dense window rows (sks_windows_dense) out.  Workers are pooled
// for the process: a parallel_* call over many files takes one per thread.
struct WindowWorker {
  int device = 0;
  hipStream_t stream = nullptr;
  sks_ctx* c = nullptr;
  uint8_t* d_in[2] = {nullptr, nullptr};
  uint64_t* d_rows[2] = {nullptr, nullptr};
  uint64_t* d_valid[2] = {nullptr, nullptr};
  uint8_t* h_in[2] = {nullptr, nullptr};
  uint64_t* h_rows[2] = {nullptr, nullptr};
  uint64_t* h_valid[2] = {nullptr, nullptr};
  hipEvent_t ev_c0[2] = {nullptr, nullptr}, ev_c1[2] = {nullptr, nullptr};  // around the D2H copies
  ~WindowWorker() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (c) sks_ctx_destroy(c);
    for (int i = 0; i < 2; ++i) {
      (void)hipFree(d_in[i]);
      (void)hipFree(d_rows[i]);
      (void)hipFree(d_valid[i]);
      (void)hipHostFree(h_in[i]);
      (void)hipHostFree(h_rows[i]);
      (void)hipHostFree(h_valid[i]);
      if (ev_c0[i]) (void)hipEventDestroy(ev_c0[i]);
      if (ev_c1[i]) (void)hipEventDestroy(ev_c1[i]);
    }
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// window starts per piece (SKS_FACADE_PIECE: bytes, for tests that cut small
// inputs into many pieces); rows are at most 4 words (w > 32)
uint64_t piece_windows() {
  static const uint64_t p = [] {
    const char* e = getenv("SKS_FACADE_PIECE");
    const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
    return v >= 64 ? v : (uint64_t)1 << 20;
  }();
  return p;
}
constexpr uint64_t kHistory = 64;  // bytes before a piece: F's 128-bit history

std::mutex g_workers_mu;
std::vector<std::unique_ptr<WindowWorker>> g_workers;  // idle workers

std::unique_ptr<WindowWorker> make_worker(int device) {
  std::unique_ptr<WindowWorker> wk(new WindowWorker);
  wk->device = device;
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipStreamCreateWithFlags(&wk->stream, hipStreamNonBlocking), "hipStreamCreate");
  check(sks_ctx_create(device, wk->stream, &wk->c));
  const uint64_t P = piece_windows();
  for (int i = 0; i < 2; ++i) {
    check_hip(hipMalloc(&wk->d_in[i], P + 2 * kHistory), "hipMalloc");
    check_hip(hipMalloc(&wk->d_rows[i], P * 4 * 8), "hipMalloc");
    check_hip(hipMalloc(&wk->d_valid[i], (P / 64 + 1) * 8), "hipMalloc");
    check_hip(hipHostMalloc(&wk->h_in[i], P + 2 * kHistory, hipHostMallocDefault), "hipHostMalloc");
    check_hip(hipHostMalloc(&wk->h_rows[i], P * 4 * 8, hipHostMallocDefault), "hipHostMalloc");
    check_hip(hipHostMalloc(&wk->h_valid[i], (P / 64 + 1) * 8, hipHostMallocDefault), "hipHostMalloc");
    check_hip(hipEventCreate(&wk->ev_c0[i]), "hipEventCreate");
    check_hip(hipEventCreate(&wk->ev_c1[i]), "hipEventCreate");
  }
  return wk;
}

struct WorkerLease {
  std::unique_ptr<WindowWorker> w;
  explicit WorkerLease(int device) {
    {
      std::lock_guard<std::mutex> lock(g_workers_mu);
      for (size_t i = 0; i < g_workers.size(); ++i)
        if (g_workers[i]->device == device) {
          w = std::move(g_workers[i]);
          g_workers.erase(g_workers.begin() + i);
          break;
        }
    }
    if (!w) w = make_worker(device);
  }
  ~WorkerLease() {
    if (!w) return;
    (void)hipSetDevice(w->device);
    if (hipStreamSynchronize(w->stream) != hipSuccess) return;  // a failed stream: drop the worker
    std::lock_guard<std::mutex> lock(g_workers_mu);
    g_workers.push_back(std::move(w));
  }
};

std::mutex g_stats_mu;
window_flow_stats g_stats{};

double ms_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

// Every window of a record stream, in order (kmer_sliding.cpp:144-185 over
// each run), as the reference's kmer objects, handed to `fn`.  The stream is
// cut into pieces of piece_windows() window starts; each piece goes to the
// worker's device with up to 64 bytes of history in front (F's 128-bit
// register) and w - 1 behind, sks_windows_dense writes every window's row,
// and the rows come back to pinned memory.  Piece k + 1's copy in, kernel and
// copy out run on the worker's stream while the host runs `fn` over piece k.
void for_each_window(const std::vector<uint8_t>& stream, const kmer_bitset& mask, int w,
                     const std::function<void(const kmer&)>& fn) {
  const auto t_begin = std::chrono::steady_clock::now();
  const uint64_t n = stream.size();
  if (w < 1 || w > 64) throw std::invalid_argument("window length must be 1..64");
  if (n < (uint64_t)w) return;
  const uint64_t starts = n - w + 1, P = piece_windows();
  const uint64_t pieces = (starts + P - 1) / P;
  const int words = sks_windows_dense_row_words(w);
  const uint64_t m[2] = {mask.lo(), mask.hi()};
  WorkerLease lease(g_device);
  WindowWorker& wk = *lease.w;
  struct Piece {
    uint64_t a, cnt;
  };
  auto issue = [&](uint64_t k) {
    const int sl = (int)(k & 1);
    const uint64_t a = k * P, cnt = std::min(P, starts - a);
    const uint64_t h = std::min<uint64_t>(a, kHistory - w);
    const uint64_t lo = a - h, hi = std::min(n, a + cnt + w - 1);
    std::memcpy(wk.h_in[sl], stream.data() + lo, hi - lo);
    check_hip(hipMemcpyAsync(wk.d_in[sl], wk.h_in[sl], hi - lo, hipMemcpyHostToDevice, wk.stream), "H2D");
    check(sks_windows_dense(wk.c, wk.d_in[sl], hi - lo, h, cnt, w, m, wk.d_rows[sl], wk.d_valid[sl]));
    check_hip(hipEventRecord(wk.ev_c0[sl], wk.stream), "hipEventRecord");
    check_hip(hipMemcpyAsync(wk.h_rows[sl], wk.d_rows[sl], cnt * words * 8, hipMemcpyDeviceToHost, wk.stream),
              "D2H");
    check_hip(hipMemcpyAsync(wk.h_valid[sl], wk.d_valid[sl], (cnt + 63) / 64 * 8, hipMemcpyDeviceToHost,
                             wk.stream), "D2H");
    check_hip(hipEventRecord(wk.ev_c1[sl], wk.stream), "hipEventRecord");
    return Piece{a, cnt};
  };
  window_flow_stats st{};
  Piece cur = issue(0);
  for (uint64_t k = 0; k < pieces; ++k) {
    const int sl = (int)(k & 1);
    const Piece nxt = k + 1 < pieces ? issue(k + 1) : Piece{0, 0};  // the slot of piece k - 1, done
    const auto t_wait = std::chrono::steady_clock::now();
    check_hip(hipEventSynchronize(wk.ev_c1[sl]), "hipEventSynchronize");
    const auto t_run = std::chrono::steady_clock::now();
    float copy_ms = 0;
    (void)hipEventElapsedTime(&copy_ms, wk.ev_c0[sl], wk.ev_c1[sl]);
    st.d2h_ms += copy_ms;
    st.d2h_bytes += cur.cnt * words * 8 + (cur.cnt + 63) / 64 * 8;
    st.wait_ms += ms_between(t_wait, t_run);
    const uint64_t* rows = wk.h_rows[sl];
    const uint64_t* valid = wk.h_valid[sl];
    for (uint64_t vw = 0; vw < (cur.cnt + 63) / 64; ++vw) {
      for (uint64_t bits = valid[vw]; bits; bits &= bits - 1) {
        const uint64_t i = vw * 64 + (uint64_t)__builtin_ctzll(bits);
        const uint64_t* r = rows + i * words;
        fn(kmer{w, kmer_bitset(r[0], r[1]), mask, kmer_bitset(r[2], words == 4 ? r[3] : 0)});
        ++st.windows;
      }
    }
    st.predicate_ms += ms_between(t_run, std::chrono::steady_clock::now());
    ++st.pieces;
    cur = nxt;
  }
  st.wall_ms = ms_between(t_begin, std::chrono::steady_clock::now());
  std::lock_guard<std::mutex> lock(g_stats_mu);
  g_stats.windows += st.windows;
  g_stats.pieces += st.pieces;
  g_stats.d2h_bytes += st.d2h_bytes;
  g_stats.d2h_ms += st.d2h_ms;
  g_stats.wait_ms += st.wait_ms;
  g_stats.predicate_ms += st.predicate_ms;
  g_stats.wall_ms += st.wall_ms;
}

std::vector<uint8_t> file_stream(const char* path) {
  FastaHandle f(path);  // strings_from_fasta's quirks; unreadable -> exit(1) like the reference
  const uint8_t* p = sks_fasta_stream(f.f);
  return std::vector<uint8_t>(p, p + sks_fasta_stream_bytes(f.f));
}

kmer_set set_from_stream(const std::vector<uint8_t>& stream, const kmer_bitset& mask, int w,
                         const sketching_condition_t& cond) {
  std::vector<kmer> kept;
  for_each_window(stream, mask, w, [&](const kmer& k) {
    if (cond(k)) kept.push_back(k);
  });
  kmer_set ks;  // kmer_set_from_fasta_file: insert_kmers of the selected list (kmer_set.cpp:54-68)
  ks.insert_kmers(kept);
  if (!ks.has_mask) {
    ks.mask = mask;
    ks.window_length = w;
    ks.has_mask = true;
  }
  return ks;
}

int g_host_threads = 0;  // set_host_threads; 0 = SKS_FACADE_THREADS, else min(16, cores)

}  // namespace

pair_flow_stats take_pair_flow_stats() {
  std::lock_guard<std::mutex> lock(g_pair_stats_mu);
  pair_flow_stats s = g_pair_stats;
  g_pair_stats = pair_flow_stats{};
  return s;
}

window_flow_stats take_window_flow_stats() {
  std::lock_guard<std::mutex> lock(g_stats_mu);
  window_flow_stats s = g_stats;
  g_stats = window_flow_stats{};
  return s;
}

void set_host_threads(int n) { g_host_threads = n > 0 ? n : 0; }

int host_threads() {
  if (g_host_threads > 0) return g_host_threads;
  if (const char* e = getenv("SKS_FACADE_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return v;
  }
  // the GPU box's share of host cores is 16 even where the machine shows more
  return std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
}

}  // namespace sks

kmer_set kmer_set_from_fasta_file(const char fasta_filename[], const kmer_bitset& mask,
                                  const int window_length, const sketching_condition_t& sketching_cond) {
  return sks::set_from_stream(sks::file_stream(fasta_filename), mask, window_length, sketching_cond);
}

std::vector<kmer_set> kmer_sets_from_fasta_files(const int num_files, char* fasta_filenames[],
                                                 const kmer_bitset& mask, const int window_length,
                                                 const sketching_condition_t& sketching_cond) {
  std::vector<kmer_set> out;
  for (int i = 0; i < num_files; ++i)
    out.push_back(kmer_set_from_fasta_file(fasta_filenames[i], mask, window_length, sketching_cond));
  return out;
}

std::vector<kmer_set> parallel_kmer_sets_from_fasta_files(const int num_files, char* fasta_filenames[],
                                                          const kmer_bitset& mask, const int window_length,
                                                          const sketching_condition_t& sketching_cond) {
  const int n = num_files > 0 ? num_files : 0;
  // open serially first so that the reference's exit(1) / error order holds
  for (int i = 0; i < n; ++i) {
    FILE* fp = fopen(fasta_filenames[i], "rb");
    if (!fp) sks::report_unreadable(fasta_filenames[i]);
    else fclose(fp);
  }
  std::vector<kmer_set> out(n);
  std::vector<std::exception_ptr> err(n);
  std::vector<std::thread> ts;
  std::atomic<int> next{0};
  // one host thread per file in flight (the reference's cilk_for over files,
  // kmer_set.cpp:124), each with its own device worker (context, stream, pinned
  // buffers): the predicates run in parallel while the devices extract windows
  const int workers = std::max(1, std::min<int>(n, sks::host_threads()));
  for (int t = 0; t < workers; ++t)
    ts.emplace_back([&]() {
      for (int i; (i = next.fetch_add(1)) < n;) {
        try {
          out[i] = kmer_set_from_fasta_file(fasta_filenames[i], mask, window_length, sketching_cond);
        } catch (...) {
          err[i] = std::current_exception();
        }
      }
    });
  for (auto& t : ts) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
  return out;
}

void nucleotide_string_list_to_kmers_by_reference(std::vector<kmer>& kmer_list,
                                                  const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketching_condition_t& sketching_cond) {
  sks::for_each_window(runs_stream(nucleotide_strings), mask, window_length, [&](const kmer& k) {
    if (sketching_cond(k)) kmer_list.push_back(k);
  });
}

std::vector<kmer> nucleotide_string_list_to_kmers(const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketching_condition_t& sketching_cond) {
  std::vector<kmer> out;
  nucleotide_string_list_to_kmers_by_reference(out, nucleotide_strings, mask, window_length,
                                               sketching_cond);
  return out;
}

// ---- pairwise -------------------------------------------------------------------------------------------
std::vector<int> compute_pairwise_kmer_set_intersections(const std::vector<kmer_set*>& kmer_sets_1,
                                                         const std::vector<kmer_set*>& kmer_sets_2) {
  if (kmer_sets_1.size() != kmer_sets_2.size())
    throw std::runtime_error("Lists of kmer sets for intersection computation have different lengths");
  std::vector<const kmer_set*> a(kmer_sets_1.begin(), kmer_sets_1.end());
  std::vector<const kmer_set*> b(kmer_sets_2.begin(), kmer_sets_2.end());
  return sks::pair_counts(a, b);
}

std::vector<int> parallel_compute_pairwise_kmer_set_intersections(
    const std::vector<kmer_set*>& kmer_sets_1, const std::vector<kmer_set*>& kmer_sets_2) {
  if (kmer_sets_1.size() != kmer_sets_2.size())
    throw std::runtime_error("Lists of kmer sets for intersection computation have different lengths");
  std::vector<const kmer_set*> a(kmer_sets_1.begin(), kmer_sets_1.end());
  std::vector<const kmer_set*> b(kmer_sets_2.begin(), kmer_sets_2.end());
  sks::PairDevices scope(sks::pool_devices());
  return sks::pair_counts(a, b);
}

// ---- fasta_processing.hpp ---------------------------------------------------------------------------------
std::vector<std::string> strings_from_fasta(const char fasta_filename[]) {
  sks::FastaHandle f(fasta_filename);
  std::vector<std::string> out(sks_fasta_num_records(f.f));
  for (uint64_t i = 0; i < out.size(); ++i) {
    const uint8_t* p;
    uint64_t n;
    sks::check(sks_fasta_record(f.f, i, &p, &n));
    out[i].assign(reinterpret_cast<const char*>(p), n);
  }
  return out;
}

void add_nucleotide_strings(std::vector<acgt_string>& return_strings, const std::string& raw_string) {
  acgt_string cur;
  for (unsigned char ch : raw_string) {
    uint8_t b = sks::nucleotide_code(ch);
    if (b & 4) {
      if (!cur.empty()) return_strings.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(b);
    }
  }
  if (!cur.empty()) return_strings.push_back(cur);
}

std::vector<acgt_string> cut_nucleotide_strings(const std::vector<std::string>& raw_strings) {
  std::vector<acgt_string> out;
  for (const std::string& s : raw_strings) add_nucleotide_strings(out, s);
  return out;
}

std::vector<acgt_string> nucleotide_strings_from_fasta_file(const char fasta_filename[]) {
  sks::FastaHandle f(fasta_filename);
  uint64_t nc = 0, nr = 0;
  sks::check(sks_fasta_runs(f.f, nullptr, nullptr, &nc, &nr));
  std::vector<uint8_t> codes(nc);
  std::vector<uint64_t> lens(nr);
  sks::check(sks_fasta_runs(f.f, codes.data(), lens.data(), &nc, &nr));
  std::vector<acgt_string> out(nr);
  uint64_t o = 0;
  for (uint64_t i = 0; i < nr; ++i) {
    out[i].assign(codes.begin() + o, codes.begin() + o + lens[i]);
    o += lens[i];
  }
  return out;
}

// ---- ani_estimator.hpp -------------------------------------------------------------------------------------
double containment(int intersection, int set_size) { return sks_containment(intersection, set_size); }
double binomial_estimator(double c, int kmer_num_ones) { return sks_binomial_estimator(c, kmer_num_ones); }
