// The reference-named C++ API (kmer.hpp, fasta_processing.hpp,
// ani_estimator.hpp) implemented on libsks.so's C ABI.  Sketching and
// intersection go to the GPU; only ingress bookkeeping, masks, hashing of
// single k-mers and the final double arithmetic run on the host — as in the
// reference, where those are host code too.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <mutex>
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

DevMem::DevMem(size_t bytes) {
  check_hip(hipSetDevice(g_device), "hipSetDevice");
  check_hip(hipMalloc(&p, bytes ? bytes : 1), "hipMalloc");
}

DevMem::~DevMem() {
  if (p) (void)hipFree(p);
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
std::vector<kmer_set> sketch_device(const uint8_t* d_seq, const std::vector<uint64_t>& off,
                                    const kmer_bitset& mask, int w, const sketch_policy& pol) {
  const size_t n_seg = off.size() - 1;
  sks_policy p{pol.kind, pol.flavour, pol.param, pol.nonce};
  uint64_t m[2] = {mask.lo(), mask.hi()};
  sks_sketch_set* set = nullptr;
  check(sks_sketch_build(ctx(), d_seq, off.back(), off.data(), (uint32_t)n_seg, w, m, &p, &set));
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
  return sketch_device(d.as<uint8_t>(), off, mask, w, pol);
}

// Raw FASTA files: the host only reads bytes; strings_from_fasta runs on the
// device (sks_fasta_parse_device) straight into the segment layout.
std::vector<kmer_set> sketch_raw_files(const std::vector<std::vector<uint8_t>>& raws,
                                       const kmer_bitset& mask, int w, const sketch_policy& pol) {
  std::vector<uint64_t> in_off(1, 0);
  for (auto& r : raws) in_off.push_back(in_off.back() + r.size());
  DevMem d_raw(in_off.back());
  for (size_t i = 0; i < raws.size(); ++i)
    if (!raws[i].empty())
      check_hip(hipMemcpy(d_raw.as<uint8_t>() + in_off[i], raws[i].data(), raws[i].size(),
                          hipMemcpyHostToDevice), "hipMemcpy H2D");
  DevMem d_stream(in_off.back() + raws.size());  // a stream is at most raw + 1 bytes
  std::vector<uint64_t> off(1, 0);
  for (size_t i = 0; i < raws.size(); ++i) {
    uint64_t nb = 0, nr = 0;
    check(sks_fasta_parse_device(ctx(), d_raw.as<uint8_t>() + in_off[i], raws[i].size(),
                                 d_stream.as<uint8_t>() + off.back(), raws[i].size() + 1, nullptr, 0,
                                 &nb, &nr));
    off.push_back(off.back() + nb);
  }
  return sketch_device(d_stream.as<uint8_t>(), off, mask, w, pol);
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

// Pair counts on the GPU for sets sharing a mask; pairs with different masks
// have no common k-mer (identity includes the mask, kmer.hpp:82-85).
std::vector<int> pair_counts(const std::vector<const kmer_set*>& a,
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
  DevMem d_words(words.size() * 8), d_starts(starts.size() * 8), d_sizes(sizes.size() * 4),
      d_a(ia.size() * 4), d_b(ib.size() * 4), d_out(a.size() * 4);
  check_hip(hipMemcpy(d_words.p, words.data(), words.size() * 8, hipMemcpyHostToDevice), "H2D");
  check_hip(hipMemcpy(d_starts.p, starts.data(), starts.size() * 8, hipMemcpyHostToDevice), "H2D");
  check_hip(hipMemcpy(d_sizes.p, sizes.data(), sizes.size() * 4, hipMemcpyHostToDevice), "H2D");
  check_hip(hipMemcpy(d_a.p, ia.data(), ia.size() * 4, hipMemcpyHostToDevice), "H2D");
  check_hip(hipMemcpy(d_b.p, ib.data(), ib.size() * 4, hipMemcpyHostToDevice), "H2D");
  std::vector<int32_t> res(a.size());
  const uint64_t n = uniq.size();
  // Pair lists that cover a large part of the n x n matrix — the reference's
  // main flow intersects generate_all_pairs_from_vector's list
  // (kmer-sketching.cpp:195-200) — are counted as the whole symmetric matrix by
  // the join kernel (sks_intersect_sym) and gathered; sparse lists go through
  // one wavefront per pair (sks_intersect_pairs).
  if (n >= 64 && n <= 16384 && a.size() * 4 >= n * n) {
    DevMem d_mat(n * n * 4);
    check(sks_intersect_sym(ctx(), d_words.as<uint64_t>(), d_starts.as<uint64_t>(),
                            d_sizes.as<uint32_t>(), ew, (uint32_t)n, 0, sks_intersect_sym_tiles((uint32_t)n),
                            d_mat.as<int32_t>()));
    check(sks_ctx_synchronize(ctx()));
    std::vector<int32_t> mat(n * n);
    check_hip(hipMemcpy(mat.data(), d_mat.p, mat.size() * 4, hipMemcpyDeviceToHost), "D2H");
    for (size_t i = 0; i < a.size(); ++i) res[i] = mat[(uint64_t)ia[i] * n + ib[i]];
  } else {
    check(sks_intersect_pairs(ctx(), d_words.as<uint64_t>(), d_starts.as<uint64_t>(),
                              d_sizes.as<uint32_t>(), ew, d_a.as<int32_t>(), d_b.as<int32_t>(),
                              a.size(), d_out.as<int32_t>()));
    check(sks_ctx_synchronize(ctx()));
    check_hip(hipMemcpy(res.data(), d_out.p, res.size() * 4, hipMemcpyDeviceToHost), "D2H");
  }
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
}

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

size_t frac_min_hash::operator()(const kmer& k) const {
  uint64_t c[2] = {k.masked_bits.lo(), k.masked_bits.hi()};
  uint64_t m[2] = {k.mask.lo(), k.mask.hi()};
  return sks_frac_min_hash(c, m, k.window_length, nonce, flavour);
}

// ---- kmer_set -------------------------------------------------------------------------------------
void kmer_set::insert_kmers(const std::vector<kmer>& kmers) {
  if (kmers.empty()) return;
  std::vector<kmer_bitset> add;
  add.reserve(kmers.size());
  for (const kmer& k : kmers) {
    if (!has_mask) {
      mask = k.mask;
      window_length = k.window_length;
      has_mask = true;
    } else if (!(k.mask == mask)) {
      throw std::runtime_error("kmer_set: k-mers with different masks cannot share a GPU sketch");
    }
    add.push_back(k.masked_bits);
  }
  std::sort(add.begin(), add.end());
  std::vector<kmer_bitset> merged;
  merged.reserve(elements.size() + add.size());
  std::merge(elements.begin(), elements.end(), add.begin(), add.end(), std::back_inserter(merged));
  merged.erase(std::unique(merged.begin(), merged.end()), merged.end());
  elements.swap(merged);
}

bool kmer_set::contains(const kmer& k) const {
  if (!has_mask || !(k.mask == mask)) return false;
  return std::binary_search(elements.begin(), elements.end(), k.masked_bits);
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
  return sks::sketch_raw_files(sks::read_files(num_files, fasta_filenames), mask, window_length,
                               policy);
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
  return compute_pairwise_kmer_set_intersections(kmer_sets_1, kmer_sets_2);
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
