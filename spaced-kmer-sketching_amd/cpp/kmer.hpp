// kmer.hpp — drop-in replacement for the reference's src/kmer.hpp
// (bensonlzl/spaced-kmer-sketching) on top of libsks.so (include/sks.h).
//
// Same names, argument meanings and error behaviour as the reference, with one
// deliberate change at the plug-in point: the reference passes the sketch
// predicate as std::function<bool(const kmer)> (kmer.hpp:93-103, :195-212),
// a host callback that cannot run inside a GPU kernel.  Here the predicate is a
// `sketch_policy` descriptor; `frac_mod_condition{frac_min_hash(1), 200}` is
// the reference's `sketching_condition` (kmer-sketching.cpp:29-34) and
// converts to it implicitly.  There is no CPU fallback: sketching and
// intersection always run on the GPU and fail loudly without one.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

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
// Sorted unique masked canonical k-mers sharing one mask (the reference's
// hash map keyed by (masked_bits, mask)).
struct kmer_set {
  int window_length = 0;
  kmer_bitset mask;
  bool has_mask = false;
  std::vector<kmer_bitset> elements;  // ascending

  // kmer.hpp:170-178 — set insert (duplicates collapse)
  void insert_kmers(const std::vector<kmer>& kmers);
  // kmer.hpp:186-189
  inline int kmer_set_size() const { return (int)elements.size(); }
  bool contains(const kmer& k) const;
};

int kmer_set_intersection(const kmer_set& ks1, const kmer_set& ks2);

// ---- sketch builders (kmer_set.cpp:54-133, kmer_sliding.cpp:199-238) ------------------------
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
// the reference's kmer_bits / masked_bits.  The predicate must be a
// per-k-mer FracMinHash condition (frac_mod_condition, or sketch_policy::frac;
// c = 1 keeps every window); a bottom-s policy throws std::invalid_argument.
// Codes are used as the reference uses them (low two bits, kmer_sliding.cpp:26-47).
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

// ---- pairwise intersections (kmer_set.cpp:143-184) ------------------------------------------------
std::vector<int> compute_pairwise_kmer_set_intersections(const std::vector<kmer_set*>& kmer_sets_1,
                                                         const std::vector<kmer_set*>& kmer_sets_2);
std::vector<int> parallel_compute_pairwise_kmer_set_intersections(
    const std::vector<kmer_set*>& kmer_sets_1, const std::vector<kmer_set*>& kmer_sets_2);

namespace sks {
// Device used by the facade (default 0); call before the first sketch.
void set_device(int device);
// Unreadable FASTA: the reference prints to stderr and exit(1)s
// (fasta_processing.cpp:86-90).  That is the default here too; pass false to
// get a std::runtime_error instead.
void set_exit_on_io_error(bool exit_on_error);
}  // namespace sks
