// ===========================================================================
// sks_oracle — CPU restatement of the reference's sketch path.
//
// TEST INFRASTRUCTURE ONLY.  Nothing in the product (libsks.so, the C++ facade,
// bench.py's measured legs) links, loads or calls this file.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only
// as the checker.
//
// What it restates (reference = bensonlzl/spaced-kmer-sketching @ 2024-10-22):
//   * FASTA ingress ............ src/fasta_processing.cpp:35-211
//   * spaced-seed mask ......... src/kmer_bitset.cpp:132-152 (libstdc++ shuffle)
//   * sliding canonical k-mers . src/kmer_sliding.cpp:26-47, 112-186, 199-238
//   * FracMinHash predicate .... src/kmer.hpp:135-149, src/kmer-sketching.cpp:29-34
//   * set / intersection ....... src/kmer.hpp:160-190, src/kmer_set.cpp:23-41
//   * containment / ANI ........ src/ani_estimation.cpp:24-42
//   * all-pairs generator ...... src/generators.hpp:44-58
//
// Pinning status:
//   * ingress + ANI: pinned against the reference's own fasta_processing.cpp /
//     ani_estimation.cpp compiled from /root/reference into oracle/_ref/ and
//     frozen as fixtures under tests/golden/.
//   * masks: pinned (libstdc++ std::shuffle + std::mt19937).
//   * the selection hash boost::hash_value(dynamic_bitset) is PARITY UNPINNED:
//     Boost is absent from the image and the reference ships no tests or
//     fixtures.  Both plausible Boost flavours are restated (B = Boost>=1.81
//     hash_mix, default; A = Boost 1.71-1.80 MurmurHash2-style combine).
// ===========================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <numeric>
#include <random>
#include <string>
#include <utility>
#include <vector>

typedef unsigned __int128 u128;

extern "C" {

// Buffer handed to Python: `data` holds `total` bytes (or u64 words, see each
// function), `lens` holds `n` lengths.  Free with ora_buf_free.
typedef struct {
  uint8_t* data;
  uint64_t* lens;
  uint64_t n;
  uint64_t total;
} ora_buf;

void ora_buf_free(ora_buf* b) {
  if (!b) return;
  free(b->data);
  free(b->lens);
  b->data = nullptr;
  b->lens = nullptr;
  b->n = b->total = 0;
}

}  // extern "C"

namespace {

// ---- ingress -------------------------------------------------------------
// fasta_processing.cpp:35-69: A/a->0 C/c->1 G/g->2 T/t->3, anything else 4.
inline uint8_t code_of(unsigned char ch) {
  switch (ch) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    case 't': case 'T': return 3;
    default: return 4;
  }
}

// fasta_processing.cpp:79-133 (getline loop, record quirks preserved).
bool records_from_fasta(const char* path, std::vector<std::string>& out) {
  std::ifstream f(path);
  if (!f.good()) return false;
  std::string name, content;
  for (std::string line; std::getline(f, line);) {
    if (line.empty() || line[0] == '>') {
      if (!name.empty()) out.push_back(content);
      if (!line.empty()) name = line.substr(1);
      content.clear();
    } else if (!name.empty()) {
      if (line.find(' ') != std::string::npos) {
        name.clear();
        content.clear();
      } else {
        content += line;
      }
    }
  }
  if (!name.empty()) out.push_back(content);
  return true;
}

// fasta_processing.cpp:144-179: split at every code-4 byte, drop empty runs.
void cut_runs(const uint8_t* s, uint64_t n, std::vector<std::vector<uint8_t>>& runs) {
  std::vector<uint8_t> cur;
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t b = code_of(s[i]);
    if (b & 4) {
      if (!cur.empty()) runs.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(b);
    }
  }
  if (!cur.empty()) runs.push_back(cur);
}

void pack_runs(const std::vector<std::vector<uint8_t>>& runs, ora_buf* out) {
  uint64_t total = 0;
  for (auto& r : runs) total += r.size();
  out->n = runs.size();
  out->total = total;
  out->data = (uint8_t*)malloc(total ? total : 1);
  out->lens = (uint64_t*)malloc(sizeof(uint64_t) * (runs.size() ? runs.size() : 1));
  uint64_t o = 0;
  for (size_t i = 0; i < runs.size(); ++i) {
    if (!runs[i].empty()) memcpy(out->data + o, runs[i].data(), runs[i].size());
    o += runs[i].size();
    out->lens[i] = runs[i].size();
  }
}

// ---- hashes ----------------------------------------------------------------
// Flavour B: Boost >= 1.81 container_hash.  hash_combine(s, v) =
// hash_mix(s + 0x9e3779b9 + v) with the 64-bit hash_mix below.
inline uint64_t mix_b(uint64_t x) {
  const uint64_t m = 0x0e9846af9b1a615dULL;
  x ^= x >> 32;
  x *= m;
  x ^= x >> 32;
  x *= m;
  x ^= x >> 28;
  return x;
}
inline uint64_t combine_b(uint64_t s, uint64_t v) { return mix_b(s + 0x9e3779b9ULL + v); }

// Flavour A: Boost 1.56-1.80 hash_combine_impl for 64-bit size_t.
inline uint64_t combine_a(uint64_t h, uint64_t k) {
  const uint64_t m = 0xc6a4a7935bd1e995ULL;
  k *= m;
  k ^= k >> 47;
  k *= m;
  h ^= k;
  h *= m;
  h += 0xe6546b64ULL;
  return h;
}

// boost::hash_value(dynamic_bitset<unsigned long>) of a 128-bit bitset:
//   res = hash_value(num_bits); hash_combine(res, m_bits)  where
//   hash_value(m_bits) = hash_range(blocks) = combine(combine(0, lo), hi).
inline uint64_t hash_bitset128(uint64_t lo, uint64_t hi, int flavour) {
  if (flavour == 0) return combine_b(128, combine_b(combine_b(0, lo), hi));
  return combine_a(128, combine_a(combine_a(0, lo), hi));
}

// kmer.hpp:141-148: fmh = H(masked) ^ H(mask) ^ hash<int>(w) ^ nonce, where
// boost::hash<int> is the identity and nonce = (int)hash<int>(n).
inline uint64_t frac_min_hash(u128 c, u128 m, int w, int64_t nonce, int flavour) {
  uint64_t hc = hash_bitset128((uint64_t)c, (uint64_t)(c >> 64), flavour);
  uint64_t hm = hash_bitset128((uint64_t)m, (uint64_t)(m >> 64), flavour);
  return hc ^ hm ^ (uint64_t)(int64_t)w ^ (uint64_t)(int64_t)(int)nonce;
}

struct Window {
  u128 f, r, c;
  uint64_t hc, fmh;
};

// kmer_sliding.cpp:112-186 restated on 128-bit integers.  Forward window
// F <<= 2 with the new base at bits 0-1 (:26-31); reverse-complement window
// R >>= 2 with comp(base) at bits 2w-2..2w-1 (:42-47); the same mask on both
// strands (:159-160); canonical = strict unsigned min, ties take R (:166-175).
template <class Fn>
void slide(const uint8_t* x, uint64_t L, int w, u128 mask, Fn&& fn) {
  if ((int64_t)L < w) return;
  u128 F = 0, R = 0;
  const int top = 2 * w - 2;
  for (int i = 0; i + 1 < w; ++i) {
    F = (F << 2) | (u128)x[i];
    R = (R >> 2) | ((u128)(x[i] ^ 3) << top);
  }
  for (uint64_t i = 0; i + w - 1 < L; ++i) {
    uint8_t b = x[i + w - 1];
    F = (F << 2) | (u128)b;
    R = (R >> 2) | ((u128)(b ^ 3) << top);
    u128 fm = F & mask, rm = R & mask;
    u128 c = (fm < rm) ? fm : rm;
    fn(F, R, c);
  }
}

void sort_unique(std::vector<u128>& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

void put_u128s(const std::vector<u128>& v, ora_buf* out) {
  out->n = v.size();
  out->total = v.size() * 2;
  out->data = (uint8_t*)malloc(16 * (v.size() ? v.size() : 1));
  out->lens = nullptr;
  uint64_t* d = (uint64_t*)out->data;
  for (size_t i = 0; i < v.size(); ++i) {
    d[2 * i] = (uint64_t)v[i];
    d[2 * i + 1] = (uint64_t)(v[i] >> 64);
  }
}

}  // namespace

extern "C" {

// ---- ingress API -------------------------------------------------------------
// Raw record strings (strings_from_fasta).  Returns 0, or 1 if the file
// cannot be opened (the reference prints to stderr and exit(1)s: :86-90).
int ora_fasta_records(const char* path, ora_buf* out) {
  std::vector<std::string> recs;
  if (!records_from_fasta(path, recs)) return 1;
  uint64_t total = 0;
  for (auto& r : recs) total += r.size();
  out->n = recs.size();
  out->total = total;
  out->data = (uint8_t*)malloc(total ? total : 1);
  out->lens = (uint64_t*)malloc(sizeof(uint64_t) * (recs.size() ? recs.size() : 1));
  uint64_t o = 0;
  for (size_t i = 0; i < recs.size(); ++i) {
    memcpy(out->data + o, recs[i].data(), recs[i].size());
    o += recs[i].size();
    out->lens[i] = recs[i].size();
  }
  return 0;
}

// ACGT runs (nucleotide_strings_from_fasta_file): codes 0..3, one byte each.
int ora_fasta_runs(const char* path, ora_buf* out) {
  std::vector<std::string> recs;
  if (!records_from_fasta(path, recs)) return 1;
  std::vector<std::vector<uint8_t>> runs;
  for (auto& r : recs) cut_runs((const uint8_t*)r.data(), r.size(), runs);
  pack_runs(runs, out);
  return 0;
}

// add_nucleotide_strings over one byte string.
int ora_cut_runs(const uint8_t* s, uint64_t n, ora_buf* out) {
  std::vector<std::vector<uint8_t>> runs;
  cut_runs(s, n, runs);
  pack_runs(runs, out);
  return 0;
}

// ---- mask ------------------------------------------------------------------
// kmer_bitset.cpp:132-152.  out[0] = bits 0..63, out[1] = bits 64..127.
int ora_mask(int w, int k, uint64_t seed, uint64_t* out) {
  if (w < 1 || w > 64 || k < 0 || k > w) return 1;
  std::vector<int> idx(w);
  std::iota(idx.begin(), idx.end(), 0);
  std::shuffle(idx.begin(), idx.end(), std::mt19937(seed));
  u128 m = 0;
  for (int i = 0; i < k; ++i) m |= (u128)3 << (2 * idx[i]);
  out[0] = (uint64_t)m;
  out[1] = (uint64_t)(m >> 64);
  return 0;
}

// ---- hashes (exposed for fixtures / tests) ---------------------------------------
uint64_t ora_hash_bitset128(uint64_t lo, uint64_t hi, int flavour) {
  return hash_bitset128(lo, hi, flavour);
}
uint64_t ora_frac_min_hash(uint64_t c_lo, uint64_t c_hi, uint64_t m_lo, uint64_t m_hi, int w,
                           int64_t nonce, int flavour) {
  return frac_min_hash(((u128)c_hi << 64) | c_lo, ((u128)m_hi << 64) | m_lo, w, nonce, flavour);
}

// Per-window dump over runs (codes, run lengths): 10 u64 per window =
// F(lo,hi) R(lo,hi) C(lo,hi) H(C) fmh run_index offset_in_run.
// F/R are reported masked to the low 2w bits (the reference's window also
// carries older bases above bit 2w, which no result depends on).
int ora_windows(const uint8_t* codes, const uint64_t* run_lens, uint64_t n_runs, int w,
                const uint64_t* mask, int64_t nonce, int flavour, ora_buf* out) {
  if (w < 1 || w > 64) return 1;
  u128 M = ((u128)mask[1] << 64) | mask[0];
  u128 wm = (w == 64) ? ~(u128)0 : (((u128)1 << (2 * w)) - 1);
  std::vector<uint64_t> rows;
  uint64_t off = 0;
  for (uint64_t r = 0; r < n_runs; ++r) {
    uint64_t i = 0;
    slide(codes + off, run_lens[r], w, M, [&](u128 F, u128 R, u128 C) {
      F &= wm;
      R &= wm;
      uint64_t hc = hash_bitset128((uint64_t)C, (uint64_t)(C >> 64), flavour);
      uint64_t f = frac_min_hash(C, M, w, nonce, flavour);
      uint64_t row[10] = {(uint64_t)F, (uint64_t)(F >> 64), (uint64_t)R, (uint64_t)(R >> 64),
                          (uint64_t)C, (uint64_t)(C >> 64), hc, f, r, i};
      rows.insert(rows.end(), row, row + 10);
      ++i;
    });
    off += run_lens[r];
  }
  out->n = rows.size() / 10;
  out->total = rows.size();
  out->data = (uint8_t*)malloc(8 * (rows.size() ? rows.size() : 1));
  out->lens = nullptr;
  if (!rows.empty()) memcpy(out->data, rows.data(), 8 * rows.size());
  return 0;
}

// nucleotide_string_list_to_kmers (kmer_sliding.cpp:112-238) with the
// FracMinHash predicate fmh % c == 0: the selected windows in order, with
// duplicates.  Each row is the reference's `kmer`: kmer_bits = the chosen
// strand's raw window register (F keeps up to 64 bases of the run, never
// cleared above bit 2w; R holds 2w bits), masked_bits = min(F & M, R & M)
// with ties to R (:159-175).  Rows: kmer_bits lo, hi, masked lo, hi, run, offset.
int ora_kmer_list(const uint8_t* codes, const uint64_t* run_lens, uint64_t n_runs, int w,
                  const uint64_t* mask, uint64_t c, int64_t nonce, int flavour, ora_buf* out) {
  if (w < 1 || w > 64 || c == 0) return 1;
  u128 M = ((u128)mask[1] << 64) | mask[0];
  std::vector<uint64_t> rows;
  uint64_t off = 0;
  for (uint64_t r = 0; r < n_runs; ++r) {
    uint64_t i = 0;
    slide(codes + off, run_lens[r], w, M, [&](u128 F, u128 R, u128 C) {
      const u128 bits = ((F & M) < (R & M)) ? F : R;
      if (frac_min_hash(C, M, w, nonce, flavour) % c == 0) {
        uint64_t row[6] = {(uint64_t)bits, (uint64_t)(bits >> 64), (uint64_t)C,
                           (uint64_t)(C >> 64), r, i};
        rows.insert(rows.end(), row, row + 6);
      }
      ++i;
    });
    off += run_lens[r];
  }
  out->n = rows.size() / 6;
  out->total = rows.size();
  out->data = (uint8_t*)malloc(8 * (rows.size() ? rows.size() : 1));
  out->lens = nullptr;
  if (!rows.empty()) memcpy(out->data, rows.data(), 8 * rows.size());
  return 0;
}

// Sketch of one genome given as runs.  kind 0 = FracMinHash (keep iff
// fmh % param == 0; kmer-sketching.cpp:30-34 with c = param), kind 1 =
// bottom-s (build-defined: the `param` distinct canonical k-mers with the
// smallest fmh, ties by k-mer value).  Output: sorted unique canonical
// k-mers as (lo, hi) u64 pairs.  *n_windows = windows hashed.
int ora_sketch(const uint8_t* codes, const uint64_t* run_lens, uint64_t n_runs, int w,
               const uint64_t* mask, int kind, uint64_t param, int64_t nonce, int flavour,
               ora_buf* out, uint64_t* n_windows) {
  if (w < 1 || w > 64 || param == 0) return 1;
  u128 M = ((u128)mask[1] << 64) | mask[0];
  const uint64_t hm = hash_bitset128(mask[0], mask[1], flavour);
  const uint64_t kconst = hm ^ (uint64_t)(int64_t)w ^ (uint64_t)(int64_t)(int)nonce;
  uint64_t nw = 0;
  std::vector<u128> keep;
  std::vector<std::pair<uint64_t, u128>> cand;
  uint64_t off = 0;
  for (uint64_t r = 0; r < n_runs; ++r) {
    slide(codes + off, run_lens[r], w, M, [&](u128, u128, u128 C) {
      ++nw;
      uint64_t f = hash_bitset128((uint64_t)C, (uint64_t)(C >> 64), flavour) ^ kconst;
      if (kind == 0) {
        if (f % param == 0) keep.push_back(C);
      } else {
        cand.emplace_back(f, C);
      }
    });
    off += run_lens[r];
  }
  if (kind == 1) {
    std::sort(cand.begin(), cand.end());
    cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
    for (size_t i = 0; i < cand.size() && keep.size() < param; ++i) keep.push_back(cand[i].second);
  }
  sort_unique(keep);
  put_u128s(keep, out);
  if (n_windows) *n_windows = nw;
  return 0;
}

// |A ∩ B| of two sorted unique (lo,hi)-pair arrays (kmer_set.cpp:23-41 counts
// the same quantity by hash probing).
int32_t ora_intersect(const uint64_t* a, uint64_t na, const uint64_t* b, uint64_t nb) {
  uint64_t i = 0, j = 0;
  int32_t n = 0;
  while (i < na && j < nb) {
    u128 x = ((u128)a[2 * i + 1] << 64) | a[2 * i];
    u128 y = ((u128)b[2 * j + 1] << 64) | b[2 * j];
    if (x < y) ++i;
    else if (y < x) ++j;
    else { ++n; ++i; ++j; }
  }
  return n;
}

// ani_estimation.cpp:24-28
double ora_containment(int intersection, int set_size) {
  if (intersection == 0) return 0;
  return ((double)intersection) / ((double)set_size);
}
// ani_estimation.cpp:38-42
double ora_binomial_estimator(double containment, int kmer_num_ones) {
  if (containment <= 0) return 0;
  return std::pow(containment, ((double)1.0) / ((double)kmer_num_ones));
}

}  // extern "C"
