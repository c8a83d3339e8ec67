// ===========================================================================
// ref_port — reference-faithful CPU port of the sketch path, used ONLY as the
// `cpu_baseline` leg of bench.py and as a second checker in tests/.
// TEST / BASELINE INFRASTRUCTURE ONLY: the product never links or calls it.
//
// The reference (bensonlzl/spaced-kmer-sketching) cannot be compiled here or
// on the GPU box: it needs Boost dynamic_bitset/container_hash and OpenCilk,
// neither of which is in the image.  This port keeps the reference's
// algorithm AND its data-structure costs so its timing is a fair stand-in:
//   * kbits: a heap-backed 128-bit bitset (std::vector<unsigned long> blocks,
//     the storage boost::dynamic_bitset<> uses), bit proxies, operator& that
//     allocates, MSB-first operator<          (kmer.hpp:27, kmer_sliding.cpp:26-47)
//   * struct kmer with three bitsets, built per window and copied into the
//     std::function predicate by value        (kmer.hpp:75-86, kmer_sliding.cpp:182-184)
//   * frac_min_hash with the Boost-flavour hash (kmer.hpp:135-149)
//   * kmer_set = std::unordered_map<kmer,int,kmer_hash> (kmer.hpp:152-190)
//   * intersection by probing the larger set (kmer_set.cpp:23-41)
//   * std::thread workers over files / over pairs standing in for cilk_for
//     (kmer_set.cpp:124, :179); a single genome runs on one worker.
// ===========================================================================
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <numeric>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace rp {

static int g_flavour = 0;  // 0 = Boost>=1.81 hash_mix, 1 = Boost 1.71-1.80

inline uint64_t mix_b(uint64_t x) {
  const uint64_t m = 0x0e9846af9b1a615dULL;
  x ^= x >> 32; x *= m; x ^= x >> 32; x *= m; x ^= x >> 28;
  return x;
}
inline uint64_t combine(uint64_t s, uint64_t v) {
  if (g_flavour == 0) return mix_b(s + 0x9e3779b9ULL + v);
  const uint64_t m = 0xc6a4a7935bd1e995ULL;
  v *= m; v ^= v >> 47; v *= m; s ^= v; s *= m; s += 0xe6546b64ULL;
  return s;
}

constexpr int KMER_BITSET_SIZE = 128;

// Heap-backed fixed 128-bit bitset with dynamic_bitset's semantics for the
// operations the path uses.
class kbits {
 public:
  std::vector<unsigned long> b;
  kbits() : b(2, 0ul) {}
  explicit kbits(int) : b(2, 0ul) {}
  struct ref {
    kbits& s; int i;
    ref& operator=(bool v) {
      unsigned long bit = 1ul << (i & 63);
      if (v) s.b[i >> 6] |= bit; else s.b[i >> 6] &= ~bit;
      return *this;
    }
  };
  ref operator[](int i) { return ref{*this, i}; }
  kbits& operator<<=(int n) {  // n < 64
    b[1] = (b[1] << n) | (b[0] >> (64 - n));
    b[0] <<= n;
    return *this;
  }
  kbits& operator>>=(int n) {
    b[0] = (b[0] >> n) | (b[1] << (64 - n));
    b[1] >>= n;
    return *this;
  }
  friend kbits operator&(const kbits& x, const kbits& y) {
    kbits r(x);
    r.b[0] &= y.b[0];
    r.b[1] &= y.b[1];
    return r;
  }
  friend bool operator<(const kbits& x, const kbits& y) {
    for (int i = 1; i >= 0; --i) {
      if (x.b[i] < y.b[i]) return true;
      if (x.b[i] > y.b[i]) return false;
    }
    return false;
  }
  friend bool operator==(const kbits& x, const kbits& y) { return x.b == y.b; }
  int count() const { return __builtin_popcountl(b[0]) + __builtin_popcountl(b[1]); }
  uint64_t hash() const {  // boost::hash_value(dynamic_bitset)
    uint64_t r = 0;
    for (unsigned long v : b) r = combine(r, v);
    return combine((uint64_t)KMER_BITSET_SIZE, r);
  }
};

struct kmer {
  int window_length;
  kbits kmer_bits;
  kbits mask;
  kbits masked_bits;
  bool operator==(const kmer& o) const { return masked_bits == o.masked_bits && mask == o.mask; }
};

struct kmer_hash {
  size_t operator()(const kmer& k) const {
    return k.masked_bits.hash() ^ k.mask.hash() ^ (size_t)k.window_length;
  }
};

struct frac_min_hash {
  int nonce;
  explicit frac_min_hash(int n) : nonce((int)(size_t)n) {}
  size_t operator()(const kmer& k) const {
    return k.masked_bits.hash() ^ k.mask.hash() ^ (size_t)k.window_length ^ (size_t)(long)nonce;
  }
};

typedef std::unordered_map<kmer, int, kmer_hash> kmer_hash_table;
struct kmer_set {
  kmer_hash_table kmer_hashes;
  void insert_kmers(const std::vector<kmer>& ks) {
    for (const kmer& k : ks) kmer_hashes[k] = 1;
  }
  int kmer_set_size() const { return (int)kmer_hashes.size(); }
};

inline void update_kmer_window(kbits& w, uint8_t b) {
  w <<= 2;
  w[0] = (b & 0x1);
  w[1] = ((b & 0x2) >> 1);
}
inline void update_complement_kmer_window(kbits& w, uint8_t b, int wl) {
  w >>= 2;
  w[2 * wl - 2] = (b & 0x1);
  w[2 * wl - 1] = ((b & 0x2) >> 1);
}

void nucleotide_string_to_kmers(std::vector<kmer>& out, const uint8_t* s, int64_t n,
                                const kbits& mask, int wl,
                                const std::function<bool(const kmer)>& cond) {
  if (n < wl) return;
  kbits cur(KMER_BITSET_SIZE), rc(KMER_BITSET_SIZE);
  for (int i = 0; i + 1 < wl; ++i) {
    update_kmer_window(cur, s[i]);
    update_complement_kmer_window(rc, s[i] ^ 0x3, wl);
  }
  for (int64_t i = 0; i + wl - 1 < n; ++i) {
    uint8_t b = s[i + wl - 1];
    update_kmer_window(cur, b);
    update_complement_kmer_window(rc, b ^ 0x3, wl);
    kbits mf = cur & mask;
    kbits mr = rc & mask;
    kbits *cb, *cm;
    if (mf < mr) { cb = &cur; cm = &mf; } else { cb = &rc; cm = &mr; }
    kmer ck{wl, *cb, mask, *cm};
    if (cond(ck)) out.push_back(ck);
  }
}

struct Sketcher {
  kbits mask;
  int w;
  frac_min_hash fmh;
  uint64_t c;
  Sketcher(uint64_t mlo, uint64_t mhi, int w_, int64_t nonce, uint64_t c_)
      : w(w_), fmh((int)nonce), c(c_) {
    mask.b[0] = mlo;
    mask.b[1] = mhi;
  }
};

kmer_set* sketch_runs(const uint8_t* codes, const uint64_t* lens, uint64_t n_runs,
                      const Sketcher& sk) {
  const frac_min_hash fmh = sk.fmh;
  const uint64_t c = sk.c;
  std::function<bool(const kmer)> cond = [fmh, c](const kmer k) { return fmh(k) % c == 0; };
  std::vector<kmer> ks;
  uint64_t off = 0;
  for (uint64_t r = 0; r < n_runs; ++r) {
    nucleotide_string_to_kmers(ks, codes + off, (int64_t)lens[r], sk.mask, sk.w, cond);
    off += lens[r];
  }
  kmer_set* s = new kmer_set();
  s->insert_kmers(ks);
  return s;
}

// Bottom-s in the reference's style (the reference has no bottom-s; this is
// what its API expresses it with): the same per-window loop and kmer objects,
// and a std::function predicate that keeps the s distinct k-mers with the
// smallest (fmh, masked bits) in a std::set plus an unordered_map for
// membership — the reference's own containers — and returns false, so the
// window list stays empty.  The kmer_set is then built from the kept k-mers.
kmer_set* bottom_runs(const uint8_t* codes, const uint64_t* lens, uint64_t n_runs,
                      const Sketcher& sk, uint64_t s) {
  const frac_min_hash fmh = sk.fmh;
  struct Key {
    uint64_t f, hi, lo;
    bool operator<(const Key& o) const {
      return f != o.f ? f < o.f : (hi != o.hi ? hi < o.hi : lo < o.lo);
    }
  };
  std::set<Key> kept;                  // the s smallest so far
  std::unordered_map<kmer, int, kmer_hash> member;
  std::function<bool(const kmer)> cond = [&](const kmer k) {
    if (s == 0) return false;
    const Key key{fmh(k), k.masked_bits.b[1], k.masked_bits.b[0]};
    if (kept.size() >= s && !(key < *kept.rbegin())) return false;
    if (member.find(k) != member.end()) return false;
    kept.insert(key);
    member[k] = 1;
    if (kept.size() > s) {
      const Key last = *kept.rbegin();
      kept.erase(std::prev(kept.end()));
      kmer gone{k.window_length, kbits(), k.mask, kbits()};
      gone.masked_bits.b[0] = last.lo;
      gone.masked_bits.b[1] = last.hi;
      member.erase(gone);
    }
    return false;
  };
  std::vector<kmer> ks;
  uint64_t off = 0;
  for (uint64_t r = 0; r < n_runs; ++r) {
    nucleotide_string_to_kmers(ks, codes + off, (int64_t)lens[r], sk.mask, sk.w, cond);
    off += lens[r];
  }
  std::vector<kmer> sel;
  for (const Key& key : kept) {
    kmer k{sk.w, kbits(), sk.mask, kbits()};
    k.masked_bits.b[0] = key.lo;
    k.masked_bits.b[1] = key.hi;
    k.kmer_bits = k.masked_bits;
    sel.push_back(k);
  }
  kmer_set* out = new kmer_set();
  out->insert_kmers(sel);
  return out;
}

int kmer_set_intersection(const kmer_set& a, const kmer_set& b) {
  if (a.kmer_set_size() < b.kmer_set_size()) return kmer_set_intersection(b, a);
  int n = 0;
  for (auto it : b.kmer_hashes)
    if (a.kmer_hashes.find(it.first) != a.kmer_hashes.end()) ++n;
  return n;
}

template <class Fn>
void parallel_for(int64_t n, int threads, Fn&& fn) {
  if (threads <= 1 || n <= 1) {
    for (int64_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<int64_t> next{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&]() {
      for (int64_t i; (i = next.fetch_add(1)) < n;) fn(i);
    });
  for (auto& t : ts) t.join();
}

// fasta_processing.cpp ingress restated inline for the file-level baseline.
bool runs_from_fasta(const char* path, std::vector<uint8_t>& codes, std::vector<uint64_t>& lens) {
  std::ifstream f(path);
  if (!f.good()) return false;
  std::vector<std::string> recs;
  std::string name, content;
  for (std::string line; std::getline(f, line);) {
    if (line.empty() || line[0] == '>') {
      if (!name.empty()) recs.push_back(content);
      if (!line.empty()) name = line.substr(1);
      content.clear();
    } else if (!name.empty()) {
      if (line.find(' ') != std::string::npos) { name.clear(); content.clear(); }
      else content += line;
    }
  }
  if (!name.empty()) recs.push_back(content);
  for (auto& r : recs) {
    uint64_t cur = 0;
    for (unsigned char ch : r) {
      uint8_t b;
      switch (ch) {
        case 'a': case 'A': b = 0; break;
        case 'c': case 'C': b = 1; break;
        case 'g': case 'G': b = 2; break;
        case 't': case 'T': b = 3; break;
        default: b = 4;
      }
      if (b & 4) {
        if (cur) lens.push_back(cur);
        cur = 0;
      } else {
        codes.push_back(b);
        ++cur;
      }
    }
    if (cur) lens.push_back(cur);
  }
  return true;
}

}  // namespace rp

extern "C" {

void rp_set_flavour(int flavour) { rp::g_flavour = flavour; }

// One genome (as runs) -> kmer_set handle.  FracMinHash keep iff fmh % c == 0.
void* rp_sketch_runs(const uint8_t* codes, const uint64_t* lens, uint64_t n_runs, int w,
                     const uint64_t* mask, uint64_t c, int64_t nonce) {
  rp::Sketcher sk(mask[0], mask[1], w, nonce, c);
  return rp::sketch_runs(codes, lens, n_runs, sk);
}

// One genome (as runs) -> bottom-s kmer_set handle (see bottom_runs).
void* rp_bottom_runs(const uint8_t* codes, const uint64_t* lens, uint64_t n_runs, int w,
                     const uint64_t* mask, uint64_t s, int64_t nonce) {
  rp::Sketcher sk(mask[0], mask[1], w, nonce, 1);
  return rp::bottom_runs(codes, lens, n_runs, sk, s);
}

// Files -> kmer_set handles, `threads` workers over files (cilk_for stand-in).
// Returns 0, or 1 if any file cannot be opened.
int rp_sketch_files(const char** paths, int n, int w, const uint64_t* mask, uint64_t c,
                    int64_t nonce, int threads, void** out) {
  rp::Sketcher sk(mask[0], mask[1], w, nonce, c);
  std::atomic<int> bad{0};
  rp::parallel_for(n, threads, [&](int64_t i) {
    std::vector<uint8_t> codes;
    std::vector<uint64_t> lens;
    if (!rp::runs_from_fasta(paths[i], codes, lens)) { bad = 1; out[i] = new rp::kmer_set(); return; }
    out[i] = rp::sketch_runs(codes.data(), lens.data(), lens.size(), sk);
  });
  return bad.load();
}

// Build a kmer_set directly from canonical values (lo,hi pairs).
void* rp_set_from_elems(const uint64_t* elems, uint64_t n, int w, const uint64_t* mask) {
  rp::kmer_set* s = new rp::kmer_set();
  std::vector<rp::kmer> ks;
  ks.reserve(n);
  for (uint64_t i = 0; i < n; ++i) {
    rp::kmer k;
    k.window_length = w;
    k.mask.b[0] = mask[0];
    k.mask.b[1] = mask[1];
    k.masked_bits.b[0] = elems[2 * i];
    k.masked_bits.b[1] = elems[2 * i + 1];
    k.kmer_bits = k.masked_bits;
    ks.push_back(k);
  }
  s->insert_kmers(ks);
  return s;
}

uint64_t rp_set_size(void* s) { return (uint64_t)((rp::kmer_set*)s)->kmer_set_size(); }

// Sorted (lo,hi) dump of a set.
void rp_set_dump(void* s, uint64_t* out) {
  std::vector<std::pair<uint64_t, uint64_t>> v;
  for (auto& kv : ((rp::kmer_set*)s)->kmer_hashes)
    v.emplace_back(kv.first.masked_bits.b[1], kv.first.masked_bits.b[0]);
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size(); ++i) {
    out[2 * i] = v[i].second;
    out[2 * i + 1] = v[i].first;
  }
}

void rp_set_free(void* s) { delete (rp::kmer_set*)s; }

// generate_all_pairs_from_vector (generators.hpp:44-58) + the parallel
// pairwise intersection (kmer_set.cpp:167-184): out[i*n+j] = |S_i ∩ S_j|.
void rp_all_pairs(void** sets, int n, int threads, int32_t* out) {
  std::vector<rp::kmer_set*> a, b;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      a.push_back((rp::kmer_set*)sets[i]);
      b.push_back((rp::kmer_set*)sets[j]);
    }
  rp::parallel_for((int64_t)a.size(), threads,
                   [&](int64_t p) { out[p] = rp::kmer_set_intersection(*a[p], *b[p]); });
}

// Pair-list form (compute_pairwise_kmer_set_intersections): only the first
// n_pairs of the i-major all-pairs order — a bounded sample for timing.
void rp_pairs_prefix(void** sets, int n, int64_t n_pairs, int threads, int32_t* out) {
  rp::parallel_for(n_pairs, threads, [&](int64_t p) {
    int64_t i = p / n, j = p % n;
    out[p] = rp::kmer_set_intersection(*(rp::kmer_set*)sets[i], *(rp::kmer_set*)sets[j]);
  });
}

}  // extern "C"
