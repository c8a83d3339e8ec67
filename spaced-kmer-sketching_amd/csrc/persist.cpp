// Persisted sketches (no reference equivalent — the
// reference re-parses and re-sketches every FASTA for each of its 62
// configurations, kmer-sketching.cpp:168).
//
// File format "SKSKETCH", little-endian, 8-byte aligned sections.
// Version 1 (one window / mask for the whole file; every C-ABI set):
//   header (96 bytes)
//     char     magic[8]   = "SKSKETCH"
//     uint32   version    = 1
//     uint32   elem_words   1 (window <= 32: one u64 per k-mer) or 2 (lo, hi)
//     int32    window       w of the spaced seed
//     int32    policy_kind  sks_policy_kind
//     int32    flavour      sks_hash_flavour
//     int32    reserved     0
//     uint64   param        c (FracMinHash) or s (bottom-s)
//     int64    nonce
//     uint64   mask_lo, mask_hi
//     uint64   n            sketches
//     uint64   total        elements over all sketches
//     uint64   names_bytes  0, or the size of the name table
//     uint64   groups       0 (version 1); the group count (version 2)
//   uint32 sizes[n]           (zero-padded to a multiple of 8 bytes)
//   uint64 windows[n]         k-mer windows hashed per genome
//   [version 2 only] group table, `groups` entries of 32 bytes:
//     uint32 set, int32 window, uint64 mask_lo, uint64 mask_hi, uint64 size
//   uint64 data[total * elem_words]   each sketch (v1) / group (v2) sorted ascending, unique
//   char   names[names_bytes] n NUL-terminated strings (when names_bytes > 0)
//   uint64 checksum           FNV-1a 64 of every byte before it
// Version 2 is what the C++ facade writes for kmer_sets the reference allows but
// version 1 cannot hold (kmer.hpp:170-178 accepts any mix of masks): a set is a
// list of (window, mask) groups in set order, sizes[i] = the sum of set i's
// group sizes, and the header's window / mask are the first group's.  The C ABI
// reads version 1 only (an sks_sketch_set has one mask).
// A reader rejects a wrong magic / version, inconsistent sizes, a truncated
// or over-long file, a checksum mismatch and unsorted sketches (SKS_E_IO).
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "sks.h"
#include "sks_api_internal.hpp"

namespace sks {

namespace {

constexpr char kMagic[8] = {'S', 'K', 'S', 'K', 'E', 'T', 'C', 'H'};
constexpr uint32_t kVersion = 1;
constexpr uint32_t kVersionGroups = 2;

struct Header {
  char magic[8];
  uint32_t version;
  uint32_t elem_words;
  int32_t window;
  int32_t policy_kind;
  int32_t flavour;
  int32_t reserved0;
  uint64_t param;
  int64_t nonce;
  uint64_t mask_lo, mask_hi;
  uint64_t n;
  uint64_t total;
  uint64_t names_bytes;
  uint64_t groups;
};
static_assert(sizeof(Header) == 96, "sketch file header layout");

struct GroupRec {
  uint32_t set;
  int32_t window;
  uint64_t mask_lo, mask_hi;
  uint64_t size;
};
static_assert(sizeof(GroupRec) == 32, "sketch file group layout");

struct Fnv {
  uint64_t h = 0xcbf29ce484222325ull;
  void add(const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
  }
};

size_t pad8(size_t x) { return (x + 7) & ~size_t(7); }

// Writes through a FILE*, hashing every byte.
struct Writer {
  FILE* f;
  Fnv fnv;
  bool ok = true;
  void put(const void* p, size_t n) {
    if (!n || !ok) return;
    fnv.add(p, n);
    ok = fwrite(p, 1, n, f) == n;
  }
};

bool less128(const uint64_t* a, const uint64_t* b, int ew) {
  if (ew == 1) return a[0] < b[0];
  return a[1] < b[1] || (a[1] == b[1] && a[0] < b[0]);
}

}  // namespace

namespace {

int write_impl(const char* path, const SketchFileMeta& meta, const std::vector<uint32_t>& sizes,
               const std::vector<uint64_t>& windows, const std::vector<SketchGroup>* groups,
               const uint64_t* data, const std::vector<std::string>& names) {
  if (!path) return fail(SKS_E_ARG, "sketch file: null path");
  if (windows.size() != sizes.size() || (!names.empty() && names.size() != sizes.size()))
    return fail(SKS_E_ARG, "sketch file: names / windows must match the number of sketches");
  Header h{};
  std::memcpy(h.magic, kMagic, 8);
  h.version = groups ? kVersionGroups : kVersion;
  h.elem_words = (uint32_t)meta.elem_words;
  h.window = meta.window;
  h.policy_kind = meta.policy.kind;
  h.flavour = meta.policy.flavour;
  h.param = meta.policy.param;
  h.nonce = meta.policy.nonce;
  h.mask_lo = meta.mask[0];
  h.mask_hi = meta.mask[1];
  h.n = sizes.size();
  for (uint32_t v : sizes) h.total += v;
  std::vector<GroupRec> recs;
  if (groups) {
    uint64_t gtotal = 0;
    for (const SketchGroup& g : *groups) {
      if (g.set >= sizes.size()) return fail(SKS_E_ARG, "sketch file: group names a missing set");
      recs.push_back(GroupRec{g.set, g.window, g.mask[0], g.mask[1], g.size});
      gtotal += g.size;
    }
    if (gtotal != h.total) return fail(SKS_E_ARG, "sketch file: group sizes do not add up");
    h.groups = recs.size();
  }
  std::string table;
  for (const std::string& s : names) {
    if (s.find('\0') != std::string::npos) return fail(SKS_E_ARG, "sketch file: name contains NUL");
    table += s;
    table.push_back('\0');
  }
  h.names_bytes = table.size();
  FILE* f = fopen(path, "wb");
  if (!f) return fail(SKS_E_IO, std::string("sketch file: cannot open ") + path + ": " + strerror(errno));
  Writer w{f};
  w.put(&h, sizeof h);
  w.put(sizes.data(), sizes.size() * 4);
  const uint64_t zero = 0;
  w.put(&zero, pad8(sizes.size() * 4) - sizes.size() * 4);
  w.put(windows.data(), windows.size() * 8);
  w.put(recs.data(), recs.size() * sizeof(GroupRec));
  w.put(data, h.total * h.elem_words * 8);
  w.put(table.data(), table.size());
  const uint64_t sum = w.fnv.h;
  if (w.ok) w.ok = fwrite(&sum, 1, 8, f) == 8;
  const bool closed = fclose(f) == 0;
  if (!w.ok || !closed) return fail(SKS_E_IO, std::string("sketch file: write failed for ") + path);
  return SKS_OK;
}

int read_impl(const char* path, SketchFileMeta& meta, std::vector<uint32_t>& sizes,
              std::vector<uint64_t>& windows, std::vector<uint64_t>& data,
              std::vector<std::string>& names, std::vector<SketchGroup>* groups,
              bool* grouped_out = nullptr) {
  if (!path) return fail(SKS_E_ARG, "sketch file: null path");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(SKS_E_IO, std::string("sketch file: cannot open ") + path);
  std::vector<uint8_t> buf;
  uint8_t tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
  const bool rd_ok = !ferror(f);
  fclose(f);
  const std::string where = std::string("sketch file ") + path + ": ";
  if (!rd_ok) return fail(SKS_E_IO, where + "read error");
  if (buf.size() < sizeof(Header) + 8) return fail(SKS_E_IO, where + "truncated");
  Header h;
  std::memcpy(&h, buf.data(), sizeof h);
  if (std::memcmp(h.magic, kMagic, 8) != 0) return fail(SKS_E_IO, where + "not a sketch file");
  if (h.version == kVersionGroups && !groups)
    return fail(SKS_E_IO, where + "version 2 (kmer_sets with several masks): load it with sks::load_kmer_sets");
  if (h.version != kVersion && h.version != kVersionGroups)
    return fail(SKS_E_IO, where + "unsupported version " + std::to_string(h.version));
  const bool grouped = h.version == kVersionGroups;
  if (h.window < 1 || h.window > 64 || h.elem_words < 1 || h.elem_words > 2 ||
      (!grouped && h.elem_words != (h.window > 32 ? 2u : 1u)))
    return fail(SKS_E_IO, where + "bad window / element width");
  if (h.n > (1ull << 32) || h.total > (1ull << 40) || (!grouped && h.groups) || h.groups > (1ull << 32))
    return fail(SKS_E_IO, where + "bad counts");
  // every region must fit in the file before any offset past it is formed: the
  // counts are bounded above, so o_names cannot wrap; names_bytes is checked
  // against the bytes left rather than added first
  const size_t o_sizes = sizeof(Header);
  const size_t o_win = o_sizes + pad8(h.n * 4);
  const size_t o_groups = o_win + h.n * 8;
  const size_t o_data = o_groups + h.groups * sizeof(GroupRec);
  const size_t o_names = o_data + h.total * h.elem_words * 8;
  const size_t body = buf.size() - 8;  // bytes before the checksum
  if (o_names > body || h.names_bytes > body - o_names)
    return fail(SKS_E_IO, where + "length does not match the header");
  const size_t o_sum = o_names + h.names_bytes;
  if (o_sum != body) return fail(SKS_E_IO, where + "length does not match the header");
  Fnv fnv;
  fnv.add(buf.data(), o_sum);
  uint64_t sum;
  std::memcpy(&sum, buf.data() + o_sum, 8);
  if (sum != fnv.h) return fail(SKS_E_IO, where + "checksum mismatch");
  sizes.resize(h.n);
  windows.resize(h.n);
  data.resize(h.total * h.elem_words);
  std::memcpy(sizes.data(), buf.data() + o_sizes, h.n * 4);
  std::memcpy(windows.data(), buf.data() + o_win, h.n * 8);
  if (!data.empty()) std::memcpy(data.data(), buf.data() + o_data, data.size() * 8);
  uint64_t total = 0;
  for (uint32_t v : sizes) total += v;
  if (total != h.total) return fail(SKS_E_IO, where + "sizes do not add up");
  const int ew = (int)h.elem_words;
  // runs that must each be sorted and unique: the sketches (v1) or the groups (v2)
  std::vector<uint64_t> runs;
  if (grouped) {
    std::vector<GroupRec> recs(h.groups);
    if (!recs.empty()) std::memcpy(recs.data(), buf.data() + o_groups, recs.size() * sizeof(GroupRec));
    std::vector<uint64_t> per_set(h.n, 0);
    groups->clear();
    uint32_t prev_set = 0;
    for (const GroupRec& r : recs) {
      if (r.set >= h.n || r.set < prev_set || r.window < 1 || r.window > 64 ||
          (r.window > 32 && ew != 2) || r.size > h.total)
        return fail(SKS_E_IO, where + "bad group table");
      prev_set = r.set;
      per_set[r.set] += r.size;
      runs.push_back(r.size);
      groups->push_back(SketchGroup{r.set, r.window, {r.mask_lo, r.mask_hi}, r.size});
    }
    for (uint64_t i = 0; i < h.n; ++i)
      if (per_set[i] != sizes[i]) return fail(SKS_E_IO, where + "group sizes do not add up");
  } else {
    runs.assign(sizes.begin(), sizes.end());
  }
  uint64_t e = 0;
  for (uint64_t v : runs) {
    for (uint64_t i = 1; i < v; ++i)
      if (!less128(&data[(e + i - 1) * ew], &data[(e + i) * ew], ew))
        return fail(SKS_E_IO, where + "a sketch is not sorted and unique");
    e += v;
  }
  names.clear();
  if (h.names_bytes) {
    const char* p = reinterpret_cast<const char*>(buf.data() + o_names);
    const char* end = p + h.names_bytes;
    if (end[-1] != '\0') return fail(SKS_E_IO, where + "name table not terminated");
    while (p < end) {
      names.emplace_back(p);
      p += names.back().size() + 1;
    }
    if (names.size() != h.n) return fail(SKS_E_IO, where + "name count does not match");
  }
  meta.window = h.window;
  meta.elem_words = ew;
  meta.mask[0] = h.mask_lo;
  meta.mask[1] = h.mask_hi;
  meta.policy = sks_policy{h.policy_kind, h.flavour, h.param, h.nonce};
  if (grouped_out) *grouped_out = grouped;
  return SKS_OK;
}

}  // namespace

int write_sketch_file(const char* path, const SketchFileMeta& meta, const std::vector<uint32_t>& sizes,
                      const std::vector<uint64_t>& windows, const uint64_t* data,
                      const std::vector<std::string>& names) {
  return write_impl(path, meta, sizes, windows, nullptr, data, names);
}

int write_sketch_file_groups(const char* path, const SketchFileMeta& meta,
                             const std::vector<uint32_t>& sizes, const std::vector<uint64_t>& windows,
                             const std::vector<SketchGroup>& groups, const uint64_t* data,
                             const std::vector<std::string>& names) {
  return write_impl(path, meta, sizes, windows, &groups, data, names);
}

int read_sketch_file(const char* path, SketchFileMeta& meta, std::vector<uint32_t>& sizes,
                     std::vector<uint64_t>& windows, std::vector<uint64_t>& data,
                     std::vector<std::string>& names) {
  return read_impl(path, meta, sizes, windows, data, names, nullptr);
}

int read_sketch_file_any(const char* path, SketchFileMeta& meta, std::vector<uint32_t>& sizes,
                         std::vector<uint64_t>& windows, std::vector<uint64_t>& data,
                         std::vector<std::string>& names, std::vector<SketchGroup>& groups,
                         bool& grouped) {
  grouped = false;
  return read_impl(path, meta, sizes, windows, data, names, &groups, &grouped);
}

}  // namespace sks

#define SKS_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return sks::fail(SKS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

namespace {

// Uploads host sketches into a new device set.
int make_device_set(int device, const sks::SketchFileMeta& meta, const std::vector<uint32_t>& sizes,
                    const std::vector<uint64_t>& windows, const uint64_t* host_data,
                    const uint64_t* device_data, std::vector<std::string> names,
                    sks_sketch_set** out) {
  sks_sketch_set* set = new (std::nothrow) sks_sketch_set();
  if (!set) return sks::fail(SKS_E_NOMEM, "out of memory");
  set->device = device;
  set->elem_words = meta.elem_words;
  set->n = (uint32_t)sizes.size();
  set->sizes = sizes;
  set->windows = windows;
  set->window = meta.window;
  set->mask[0] = meta.mask[0];
  set->mask[1] = meta.mask[1];
  set->policy = meta.policy;
  set->names = std::move(names);
  set->starts.resize(set->n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < set->n; ++i) {
    set->starts[i] = total;
    total += sizes[i];
  }
  auto bail = [&](const char* what) {
    sks_sketch_set_free(set);
    return sks::fail(SKS_E_HIP, std::string("sketch set: ") + what);
  };
  const size_t data_bytes = std::max<uint64_t>(total * meta.elem_words, 1) * 8;
  if (hipMalloc(reinterpret_cast<void**>(&set->d_data), data_bytes) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&set->d_starts), std::max<uint32_t>(set->n, 1) * 8) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&set->d_sizes), std::max<uint32_t>(set->n, 1) * 4) != hipSuccess)
    return bail("hipMalloc failed");
  const size_t words = total * meta.elem_words;
  if (words && host_data &&
      hipMemcpy(set->d_data, host_data, words * 8, hipMemcpyHostToDevice) != hipSuccess)
    return bail("upload failed");
  if (words && device_data &&
      hipMemcpy(set->d_data, device_data, words * 8, hipMemcpyDeviceToDevice) != hipSuccess)
    return bail("device copy failed");
  if (set->n && (hipMemcpy(set->d_starts, set->starts.data(), set->n * 8, hipMemcpyHostToDevice) != hipSuccess ||
                 hipMemcpy(set->d_sizes, sizes.data(), set->n * 4, hipMemcpyHostToDevice) != hipSuccess))
    return bail("metadata upload failed");
  *out = set;
  return SKS_OK;
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" {

int sks_sketch_set_info(const sks_sketch_set* set, sks_sketch_info* info) {
  if (!set || !info) return sks::fail(SKS_E_ARG, "sks_sketch_set_info: null argument");
  info->window = set->window;
  info->elem_words = set->elem_words;
  info->mask[0] = set->mask[0];
  info->mask[1] = set->mask[1];
  info->policy = set->policy;
  info->n = set->n;
  info->has_names = set->names.empty() ? 0 : 1;
  return SKS_OK;
}

const char* sks_sketch_set_name(const sks_sketch_set* set, uint32_t i) {
  if (!set || i >= set->names.size()) return nullptr;
  return set->names[i].c_str();
}

int sks_sketch_set_set_names(sks_sketch_set* set, const char* const* names) {
  if (!set) return sks::fail(SKS_E_ARG, "sks_sketch_set_set_names: null set");
  std::vector<std::string> v;
  if (names)
    for (uint32_t i = 0; i < set->n; ++i) {
      if (!names[i]) return sks::fail(SKS_E_ARG, "sks_sketch_set_set_names: null name");
      v.emplace_back(names[i]);
    }
  set->names = std::move(v);
  return SKS_OK;
}

int sks_sketch_set_save(const sks_sketch_set* set, const char* path) {
  if (!set || !path) return sks::fail(SKS_E_ARG, "sks_sketch_set_save: null argument");
  DevGuard g(set->device);
  uint64_t total = 0;
  for (uint32_t v : set->sizes) total += v;
  std::vector<uint64_t> host(total * set->elem_words);
  if (!host.empty())
    SKS_HIP(hipMemcpy(host.data(), set->d_data, host.size() * 8, hipMemcpyDeviceToHost));
  sks::SketchFileMeta meta;
  meta.window = set->window;
  meta.elem_words = set->elem_words;
  meta.mask[0] = set->mask[0];
  meta.mask[1] = set->mask[1];
  meta.policy = set->policy;
  return sks::write_sketch_file(path, meta, set->sizes, set->windows, host.data(), set->names);
}

int sks_sketch_set_load(sks_ctx* ctx, const char* path, sks_sketch_set** out) {
  if (!ctx || !path || !out) return sks::fail(SKS_E_ARG, "sks_sketch_set_load: null argument");
  *out = nullptr;
  sks::SketchFileMeta meta;
  std::vector<uint32_t> sizes;
  std::vector<uint64_t> windows, data;
  std::vector<std::string> names;
  int rc = sks::read_sketch_file(path, meta, sizes, windows, data, names);
  if (rc != SKS_OK) return rc;
  const int device = sks_ctx_device(ctx);
  DevGuard g(device);
  return make_device_set(device, meta, sizes, windows, data.data(), nullptr, std::move(names), out);
}

int sks_sketch_set_concat(sks_ctx* ctx, const sks_sketch_set* const* sets, uint32_t n_sets,
                          sks_sketch_set** out) {
  if (!ctx || !out || (n_sets && !sets)) return sks::fail(SKS_E_ARG, "sks_sketch_set_concat: null argument");
  *out = nullptr;
  if (n_sets == 0) return sks::fail(SKS_E_ARG, "sks_sketch_set_concat: no sets");
  const sks_sketch_set* a = sets[0];
  bool names = true;
  for (uint32_t i = 0; i < n_sets; ++i) {
    const sks_sketch_set* b = sets[i];
    if (!b) return sks::fail(SKS_E_ARG, "sks_sketch_set_concat: null set");
    if (b->window != a->window || b->elem_words != a->elem_words || b->mask[0] != a->mask[0] ||
        b->mask[1] != a->mask[1] || b->policy.kind != a->policy.kind ||
        b->policy.param != a->policy.param || b->policy.nonce != a->policy.nonce ||
        b->policy.flavour != a->policy.flavour)
      return sks::fail(SKS_E_ARG, "sks_sketch_set_concat: sets differ in window, mask or policy");
    names = names && (b->names.size() == b->n);
  }
  const int device = sks_ctx_device(ctx);
  DevGuard g(device);
  std::vector<uint32_t> sizes;
  std::vector<uint64_t> windows;
  std::vector<std::string> all_names;
  uint64_t total = 0;
  for (uint32_t i = 0; i < n_sets; ++i) {
    sizes.insert(sizes.end(), sets[i]->sizes.begin(), sets[i]->sizes.end());
    windows.insert(windows.end(), sets[i]->windows.begin(), sets[i]->windows.end());
    if (names) all_names.insert(all_names.end(), sets[i]->names.begin(), sets[i]->names.end());
    for (uint32_t v : sets[i]->sizes) total += v;
  }
  const int ew = a->elem_words;
  uint64_t* staged = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&staged), std::max<uint64_t>(total * ew, 1) * 8) != hipSuccess)
    return sks::fail(SKS_E_HIP, "sks_sketch_set_concat: hipMalloc failed");
  uint64_t at = 0;
  for (uint32_t i = 0; i < n_sets; ++i) {
    uint64_t words = 0;
    for (uint32_t v : sets[i]->sizes) words += (uint64_t)v * ew;
    if (words && hipMemcpy(staged + at, sets[i]->d_data, words * 8, hipMemcpyDefault) != hipSuccess) {
      (void)hipFree(staged);
      return sks::fail(SKS_E_HIP, "sks_sketch_set_concat: copy failed");
    }
    at += words;
  }
  sks::SketchFileMeta meta;
  meta.window = a->window;
  meta.elem_words = ew;
  meta.mask[0] = a->mask[0];
  meta.mask[1] = a->mask[1];
  meta.policy = a->policy;
  const int rc = make_device_set(device, meta, sizes, windows, nullptr, staged, std::move(all_names), out);
  (void)hipFree(staged);
  return rc;
}

}  // extern "C"
