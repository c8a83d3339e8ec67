// kmer.hpp — drop-in replacement for the reference's src/kmer.hpp
// (bensonlzl/spaced-kmer-sketching) on top of libsks.so (include/sks.h).
//
// Same names, argument meanings and error behaviour as the reference.  The
// plug-in point keeps the reference's signature: every builder takes
// std::function<bool(const kmer)> sketching_cond (kmer.hpp:93-103, :195-212),
// called once per window in window order like kmer_sliding.cpp:183.  The GPU
// extracts every window (canonical masked k-mer, kmer_bits) and the host
// predicate filters them.  For the FracMinHash predicate the selection itself
// runs on the GPU: pass `frac_mod_condition{frac_min_hash(1), 200}` (the
// reference's `sketching_condition`, kmer-sketching.cpp:29-34) or a
// `sketch_policy` (FracMinHash or bottom-s descriptor) instead of a callback.
// There is no CPU fallback: without a GPU every builder throws.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <iterator>
#include <optional>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "stl_includes.hpp"  // kmer.hpp:12 — the reference's transitive STL surface
#include "logging.hpp"       // kmer.hpp:21
#include "sks.h"

// ---- constants (kmer.hpp:37-54) --------------------------------------------------------
constexpr int LOG_KMER_BITSET_SIZE = 7;
constexpr int PARALLEL_DISABLE = 0;
constexpr int NUCLEOTIDE_BIT_SIZE = 2;
constexpr int KMER_BITSET_SIZE = (1 << LOG_KMER_BITSET_SIZE);
constexpr int MAX_KMER_LENGTH = (KMER_BITSET_SIZE / NUCLEOTIDE_BIT_SIZE);

// ---- kmer_bitset (kmer.hpp:27: boost::dynamic_bitset<> of 128 bits) -----------------------
// A fixed 128-bit value with the dynamic_bitset operations the reference uses.
// Bit 0 is the least significant bit; operator< compares as an unsigned
// 128-bit integer (dynamic_bitset compares blocks from the most significant).
class kmer_bitset {
 public:
  kmer_bitset() = default;
  explicit kmer_bitset(std::size_t num_bits) { (void)num_bits; }
  kmer_bitset(uint64_t lo, uint64_t hi) : lo_(lo), hi_(hi) {}

  class reference {
   public:
    reference(kmer_bitset& b, int i) : b_(b), i_(i) {}
    reference& operator=(bool v) { b_.set(i_, v); return *this; }
    reference& operator=(const reference& r) { b_.set(i_, bool(r)); return *this; }
    operator bool() const { return b_.test(i_); }
    bool operator~() const { return !b_.test(i_); }
   private:
    kmer_bitset& b_;
    int i_;
  };

  std::size_t size() const { return KMER_BITSET_SIZE; }
  std::size_t num_blocks() const { return 2; }
  uint64_t lo() const { return lo_; }
  uint64_t hi() const { return hi_; }

  bool test(std::size_t i) const { return i < 64 ? (lo_ >> i) & 1 : (hi_ >> (i - 64)) & 1; }
  bool operator[](std::size_t i) const { return test(i); }
  reference operator[](std::size_t i) { return reference(*this, (int)i); }
  kmer_bitset& set(std::size_t i, bool v = true) {
    uint64_t& w = i < 64 ? lo_ : hi_;
    uint64_t bit = 1ull << (i & 63);
    w = v ? (w | bit) : (w & ~bit);
    return *this;
  }
  kmer_bitset& set() { lo_ = hi_ = ~0ull; return *this; }
  kmer_bitset& reset(std::size_t i) { return set(i, false); }
  kmer_bitset& reset() { lo_ = hi_ = 0; return *this; }
  kmer_bitset& flip() { lo_ = ~lo_; hi_ = ~hi_; return *this; }
  kmer_bitset& flip(std::size_t i) { return set(i, !test(i)); }
  std::size_t count() const { return __builtin_popcountll(lo_) + __builtin_popcountll(hi_); }
  bool any() const { return lo_ | hi_; }
  bool none() const { return !any(); }

  kmer_bitset& operator<<=(std::size_t n) {
    if (n >= 128) { lo_ = hi_ = 0; }
    else if (n >= 64) { hi_ = lo_ << (n - 64); lo_ = 0; }
    else if (n) { hi_ = (hi_ << n) | (lo_ >> (64 - n)); lo_ <<= n; }
    return *this;
  }
  kmer_bitset& operator>>=(std::size_t n) {
    if (n >= 128) { lo_ = hi_ = 0; }
    else if (n >= 64) { lo_ = hi_ >> (n - 64); hi_ = 0; }
    else if (n) { lo_ = (lo_ >> n) | (hi_ << (64 - n)); hi_ >>= n; }
    return *this;
  }
  kmer_bitset operator<<(std::size_t n) const { kmer_bitset r(*this); return r <<= n; }
  kmer_bitset operator>>(std::size_t n) const { kmer_bitset r(*this); return r >>= n; }
  kmer_bitset& operator&=(const kmer_bitset& o) { lo_ &= o.lo_; hi_ &= o.hi_; return *this; }
  kmer_bitset& operator|=(const kmer_bitset& o) { lo_ |= o.lo_; hi_ |= o.hi_; return *this; }
  kmer_bitset& operator^=(const kmer_bitset& o) { lo_ ^= o.lo_; hi_ ^= o.hi_; return *this; }
  kmer_bitset operator~() const { return kmer_bitset(~lo_, ~hi_); }
  friend kmer_bitset operator&(kmer_bitset a, const kmer_bitset& b) { return a &= b; }
  friend kmer_bitset operator|(kmer_bitset a, const kmer_bitset& b) { return a |= b; }
  friend kmer_bitset operator^(kmer_bitset a, const kmer_bitset& b) { return a ^= b; }
  friend bool operator==(const kmer_bitset& a, const kmer_bitset& b) { return a.lo_ == b.lo_ && a.hi_ == b.hi_; }
  friend bool operator!=(const kmer_bitset& a, const kmer_bitset& b) { return !(a == b); }
  friend bool operator<(const kmer_bitset& a, const kmer_bitset& b) {
    return a.hi_ < b.hi_ || (a.hi_ == b.hi_ && a.lo_ < b.lo_);
  }
  friend bool operator>(const kmer_bitset& a, const kmer_bitset& b) { return b < a; }
  friend bool operator<=(const kmer_bitset& a, const kmer_bitset& b) { return !(b < a); }
  friend bool operator>=(const kmer_bitset& a, const kmer_bitset& b) { return !(a < b); }
  // dynamic_bitset stream format: most significant bit first, one char per bit.
  std::string to_string() const {
    std::string s(KMER_BITSET_SIZE, '0');
    for (int i = 0; i < KMER_BITSET_SIZE; ++i)
      if (test(i)) s[KMER_BITSET_SIZE - 1 - i] = '1';
    return s;
  }
  friend std::ostream& operator<<(std::ostream& os, const kmer_bitset& b) { return os << b.to_string(); }

 private:
  uint64_t lo_ = 0, hi_ = 0;
};

// ---- mask helpers (kmer.hpp:57-64, kmer_bitset.cpp) ---------------------------------------
void initialise_contiguous_kmer_array();
kmer_bitset contiguous_kmer(const int kmer_length);  // throws std::runtime_error if > 64
void initialise_reversing_kmer_array();
kmer_bitset reverse_kmer_bitset(const kmer_bitset& kbs);
kmer_bitset generate_random_spaced_seed_mask(const int window_size, const int kmer_size,
                                             size_t random_seed = 0);

// ---- kmer (kmer.hpp:75-86) ----------------------------------------------------------------
struct kmer {
  int window_length;
  kmer_bitset kmer_bits;
  kmer_bitset mask;
  kmer_bitset masked_bits;
  bool operator==(const kmer& other) const {
    return (masked_bits == other.masked_bits) && (mask == other.mask);
  }
};

// kmers.cpp:16-35 (legacy canonicalisation; host)
kmer reverse_complement(kmer k);
kmer canonical_kmer(kmer k);

// ---- hashes (kmer.hpp:113-149) --------------------------------------------------------------
// Hash flavour of boost::hash_value(dynamic_bitset); see DESIGN.md.
namespace sks {
void set_hash_flavour(int flavour);  // SKS_HASH_BOOST_MIX (default) or SKS_HASH_BOOST_LEGACY
int hash_flavour();
uint64_t bitset_hash(const kmer_bitset& b);
}  // namespace sks

// The host-predicate flow (every builder taking a std::function: the GPU
// extracts every window, the host predicate selects): totals since the last
// take, summed over the worker threads of a parallel_* call.  d2h_ms sums the
// device-to-host copy durations (HIP events), wait_ms the host's waits for a
// piece, predicate_ms the host time spent in the predicate loops.
namespace sks {
struct window_flow_stats {
  uint64_t windows = 0, pieces = 0, d2h_bytes = 0;
  double d2h_ms = 0, wait_ms = 0, predicate_ms = 0, wall_ms = 0;
};
window_flow_stats take_window_flow_stats();
// Pair counts on the GPU ([parallel_]compute_pairwise_kmer_set_intersections):
// bytes moved since the last take — the sketches cross PCIe once (h2d), reach
// the other pool devices device to device (d2d), and each device sends back
// only its own tiles (d2h).
struct pair_flow_stats {
  uint64_t calls = 0, devices = 0, h2d_bytes = 0, d2d_bytes = 0, d2h_bytes = 0;
};
pair_flow_stats take_pair_flow_stats();
// Host threads of parallel_kmer_sets_from_fasta_files with a std::function
// predicate (one device worker each); 0 restores the default
// (SKS_FACADE_THREADS, else min(16, cores)).
void set_host_threads(int n);
int host_threads();
}  // namespace sks

struct kmer_hash {
  size_t operator()(const kmer& k) const {
    return sks::bitset_hash(k.masked_bits) ^ sks::bitset_hash(k.mask) ^ (size_t)k.window_length;
  }
};

struct frac_min_hash {
  int nonce;
  int flavour;
  explicit frac_min_hash(int n) : nonce((int)(size_t)n), flavour(sks::hash_flavour()) {}
  size_t operator()(const kmer& k) const;
};

// ---- the device-side sketch predicate ---------------------------------------------------------
struct sketch_policy {
  int kind = SKS_FRAC_MOD;
  uint64_t param = 200;
  int64_t nonce = 1;
  int flavour = SKS_HASH_BOOST_MIX;
  static sketch_policy frac(uint64_t c, int64_t nonce = 1, int flavour = sks::hash_flavour()) {
    return sketch_policy{SKS_FRAC_MOD, c, nonce, flavour};
  }
  static sketch_policy bottom(uint64_t s, int64_t nonce = 1, int flavour = sks::hash_flavour()) {
    return sketch_policy{SKS_BOTTOM_S, s, nonce, flavour};
  }
};

// `fmh(k) % c == 0` — the reference's sketching_condition with c = 200
// (kmer-sketching.cpp:29-34) is frac_mod_condition{frac_min_hash(1), 200}.
struct frac_mod_condition {
  frac_min_hash fmh;
  uint64_t c;
  bool operator()(const kmer& k) const { return fmh(k) % c == 0; }
  operator sketch_policy() const { return sketch_policy{SKS_FRAC_MOD, c, fmh.nonce, fmh.flavour}; }
};

// ---- kmer_set (kmer.hpp:152-190) ---------------------------------------------------------------
// The reference keys its set by (masked_bits, mask) in an unordered_map
// (kmer.hpp:152, :170-178).  Here a set is one sorted array of masked bits per
// mask: `elements` under `mask` (every set the builders make has one mask),
// plus `other_masks` when k-mers with further masks were inserted.
struct kmer_set;

// Read-only view with the reference's kmer_set::kmer_hashes interface (an
// unordered_map<kmer, int, kmer_hash> whose values are all 1): size(), empty(),
// count(), contains(), at(), find(), and iteration over std::pair<const kmer, int>.
// The kmer a view yields has kmer_bits = masked_bits (the reference keeps the
// unmasked window of the first insertion there, which no result depends on).
class kmer_hash_view {
 public:
  using key_type = kmer;
  using mapped_type = int;
  using value_type = std::pair<const kmer, int>;
  using size_type = std::size_t;

  class const_iterator {
   public:
    using iterator_category = std::forward_iterator_tag;
    using value_type = kmer_hash_view::value_type;
    using difference_type = std::ptrdiff_t;
    using pointer = const value_type*;
    using reference = const value_type&;
    const_iterator() = default;
    reference operator*() const { return *cur_; }
    pointer operator->() const { return &*cur_; }
    const_iterator& operator++() { ++e_; settle(); return *this; }
    const_iterator operator++(int) { const_iterator t = *this; ++*this; return t; }
    friend bool operator==(const const_iterator& a, const const_iterator& b) {
      return a.s_ == b.s_ && a.g_ == b.g_ && a.e_ == b.e_;
    }
    friend bool operator!=(const const_iterator& a, const const_iterator& b) { return !(a == b); }

   private:
    friend class kmer_hash_view;
    const_iterator(const kmer_set* s, std::size_t g, std::size_t e) : s_(s), g_(g), e_(e) { settle(); }
    void settle();  // skip empty groups; materialise the current pair
    const kmer_set* s_ = nullptr;
    std::size_t g_ = 0, e_ = 0;  // group (0 = elements, i = other_masks[i - 1]), element
    std::optional<value_type> cur_;
  };
  using iterator = const_iterator;

  std::size_t size() const;
  bool empty() const { return size() == 0; }
  std::size_t count(const kmer& k) const;
  bool contains(const kmer& k) const { return count(k) != 0; }
  int at(const kmer& k) const;  // 1, or std::out_of_range like unordered_map::at
  const_iterator find(const kmer& k) const;
  const_iterator begin() const;
  const_iterator end() const;
  const_iterator cbegin() const { return begin(); }
  const_iterator cend() const { return end(); }

 private:
  friend struct kmer_set;
  explicit kmer_hash_view(const kmer_set* s) : s_(s) {}
  const kmer_set* s_;
};

struct kmer_set {
  int window_length = 0;
  kmer_bitset mask;
  bool has_mask = false;
  std::vector<kmer_bitset> elements;  // masked bits under `mask`, ascending, unique
  struct mask_group {
    int window_length;
    kmer_bitset mask;
    std::vector<kmer_bitset> elements;  // ascending, unique
  };
  std::vector<mask_group> other_masks;  // further masks, in first-insertion order
  kmer_hash_view kmer_hashes{this};     // kmer.hpp:162

  kmer_set() = default;
  kmer_set(const kmer_set& o)
      : window_length(o.window_length), mask(o.mask), has_mask(o.has_mask), elements(o.elements),
        other_masks(o.other_masks) {}
  kmer_set(kmer_set&& o) noexcept
      : window_length(o.window_length), mask(o.mask), has_mask(o.has_mask),
        elements(std::move(o.elements)), other_masks(std::move(o.other_masks)) {}
  kmer_set& operator=(const kmer_set& o) {
    window_length = o.window_length; mask = o.mask; has_mask = o.has_mask;
    elements = o.elements; other_masks = o.other_masks;
    return *this;
  }
  kmer_set& operator=(kmer_set&& o) noexcept {
    window_length = o.window_length; mask = o.mask; has_mask = o.has_mask;
    elements = std::move(o.elements); other_masks = std::move(o.other_masks);
    return *this;
  }

  // kmer.hpp:170-178 — set insert (duplicates collapse; any mix of masks)
  void insert_kmers(const std::vector<kmer>& kmers);
  // kmer.hpp:186-189
  int kmer_set_size() const;
  bool contains(const kmer& k) const;
  // the sorted masked bits held under mask m (nullptr if none)
  const std::vector<kmer_bitset>* elements_for(const kmer_bitset& m) const;
};

int kmer_set_intersection(const kmer_set& ks1, const kmer_set& ks2);

// ---- sketch builders (kmer_set.cpp:54-133, kmer_sliding.cpp:199-238) ------------------------
// The reference's plug-in point: any std::function<bool(const kmer)> predicate,
// called for every window of every run in order (kmer_sliding.cpp:144-185),
// with the reference's kmer (window_length, kmer_bits, mask, masked_bits).
using sketching_condition_t = std::function<bool(const kmer)>;

kmer_set kmer_set_from_fasta_file(const char fasta_filename[], const kmer_bitset& mask,
                                  const int window_length, const sketching_condition_t& sketching_cond);
std::vector<kmer_set> kmer_sets_from_fasta_files(const int num_files, char* fasta_filenames[],
                                                 const kmer_bitset& mask, const int window_length,
                                                 const sketching_condition_t& sketching_cond);
// One host thread per file (the reference's cilk_for, kmer_set.cpp:124): the
// predicate is called concurrently for different files and must be thread-safe,
// as in the reference.
std::vector<kmer_set> parallel_kmer_sets_from_fasta_files(const int num_files, char* fasta_filenames[],
                                                          const kmer_bitset& mask, const int window_length,
                                                          const sketching_condition_t& sketching_cond);
std::vector<kmer> nucleotide_string_list_to_kmers(const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketching_condition_t& sketching_cond);
void nucleotide_string_list_to_kmers_by_reference(std::vector<kmer>& kmer_list,
                                                  const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketching_condition_t& sketching_cond);

// GPU-selected forms: a sketch_policy descriptor (FracMinHash or bottom-s), or
// frac_mod_condition (converted to its FracMinHash descriptor).
kmer_set kmer_set_from_fasta_file(const char fasta_filename[], const kmer_bitset& mask,
                                  const int window_length, const sketch_policy& policy);
std::vector<kmer_set> kmer_sets_from_fasta_files(const int num_files, char* fasta_filenames[],
                                                 const kmer_bitset& mask, const int window_length,
                                                 const sketch_policy& policy);
// Files are read on worker threads; parsing (sks_fasta_parse_device) and
// sketching run on the GPU, all files in one batched build.
std::vector<kmer_set> parallel_kmer_sets_from_fasta_files(const int num_files,
                                                          char* fasta_filenames[],
                                                          const kmer_bitset& mask,
                                                          const int window_length,
                                                          const sketch_policy& policy);
// nucleotide_string_list_to_kmers[_by_reference] (kmer_sliding.cpp:199-238):
// every selected window of every run, in order, duplicates kept, each with
// the reference's kmer_bits / masked_bits.  The policy must be a per-k-mer
// FracMinHash condition (c = 1 keeps every window); a bottom-s policy throws
// std::invalid_argument.  Codes act through their low two bits (kmer_sliding.cpp:26-47).
std::vector<kmer> nucleotide_string_list_to_kmers(const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketch_policy& sketching_cond);
void nucleotide_string_list_to_kmers_by_reference(std::vector<kmer>& kmer_list,
                                                  const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                                  const kmer_bitset& mask, const int window_length,
                                                  const sketch_policy& sketching_cond);
// The set of k-mers nucleotide_string_list_to_kmers selects from these runs
// (duplicates collapsed).
kmer_set nucleotide_string_list_to_kmer_set(const std::vector<std::vector<uint8_t>>& nucleotide_strings,
                                            const kmer_bitset& mask, const int window_length,
                                            const sketch_policy& policy);

// frac_mod_condition is both callable and a descriptor; these exact overloads
// pick the GPU-selected form.
inline kmer_set kmer_set_from_fasta_file(const char f[], const kmer_bitset& m, const int w,
                                         const frac_mod_condition& c) {
  return kmer_set_from_fasta_file(f, m, w, sketch_policy(c));
}
inline std::vector<kmer_set> kmer_sets_from_fasta_files(const int n, char* f[], const kmer_bitset& m,
                                                        const int w, const frac_mod_condition& c) {
  return kmer_sets_from_fasta_files(n, f, m, w, sketch_policy(c));
}
inline std::vector<kmer_set> parallel_kmer_sets_from_fasta_files(const int n, char* f[], const kmer_bitset& m,
                                                                 const int w, const frac_mod_condition& c) {
  return parallel_kmer_sets_from_fasta_files(n, f, m, w, sketch_policy(c));
}
inline std::vector<kmer> nucleotide_string_list_to_kmers(const std::vector<std::vector<uint8_t>>& r,
                                                         const kmer_bitset& m, const int w,
                                                         const frac_mod_condition& c) {
  return nucleotide_string_list_to_kmers(r, m, w, sketch_policy(c));
}
inline void nucleotide_string_list_to_kmers_by_reference(std::vector<kmer>& out,
                                                         const std::vector<std::vector<uint8_t>>& r,
                                                         const kmer_bitset& m, const int w,
                                                         const frac_mod_condition& c) {
  nucleotide_string_list_to_kmers_by_reference(out, r, m, w, sketch_policy(c));
}

// ---- pairwise intersections (kmer_set.cpp:143-184) ------------------------------------------------
std::vector<int> compute_pairwise_kmer_set_intersections(const std::vector<kmer_set*>& kmer_sets_1,
                                                         const std::vector<kmer_set*>& kmer_sets_2);
std::vector<int> parallel_compute_pairwise_kmer_set_intersections(
    const std::vector<kmer_set*>& kmer_sets_1, const std::vector<kmer_set*>& kmer_sets_2);

namespace sks {
// Device used by the facade (default 0); call before the first sketch.
void set_device(int device);
// Devices the parallel_* entry points spread their work over (the reference's
// cilk_for over files and pairs, kmer_set.cpp:112-133,167-184, mapped onto the
// node's GPUs).  Default: every visible device, or the one set_device chose;
// the environment variable SKS_FACADE_DEVICES ("0,1,..."; a device may repeat,
// giving it several contexts) overrides the default.  An empty list restores it.
void set_devices(const std::vector<int>& devices);
std::vector<int> parallel_devices();
// Unreadable FASTA: the reference prints to stderr and exit(1)s
// (fasta_processing.cpp:86-90).  That is the default here too; pass false to
// get a std::runtime_error instead.
void set_exit_on_io_error(bool exit_on_error);
}  // namespace sks
