// Drives the reference-named C++ facade the way the reference's own driver
// does (kmer-sketching.cpp:151-212) and prints JSON for tests/test_facade.py.
//   test_facade sketch <w> <k> <mask_seed> <c|s> <frac|bottom> <file>...
//   test_facade errors
//   test_facade missing <file>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "ani_estimator.hpp"
#include "fasta_processing.hpp"
#include "generators.hpp"
#include "kmer.hpp"
#include "sketch_io.hpp"
#include "sweep.hpp"

static void hexset(const kmer_set& ks) {
  std::printf("[");
  for (size_t i = 0; i < ks.elements.size(); ++i) {
    const kmer_bitset& e = ks.elements[i];
    std::printf("%s\"%016llx%016llx\"", i ? "," : "", (unsigned long long)e.hi(),
                (unsigned long long)e.lo());
  }
  std::printf("]");
}

static int sketch(int argc, char** argv) {
  const int w = std::atoi(argv[2]), k = std::atoi(argv[3]);
  const size_t seed = std::strtoull(argv[4], nullptr, 10);
  const uint64_t param = std::strtoull(argv[5], nullptr, 10);
  const bool bottom = std::string(argv[6]) == "bottom";
  const int n = argc - 7;
  char** files = argv + 7;

  kmer_bitset mask = generate_random_spaced_seed_mask(w, k, seed);
  const int kmer_num_indices = (int)(mask.count() / NUCLEOTIDE_BIT_SIZE);
  frac_min_hash fmh(1);
  sketch_policy policy = bottom ? sketch_policy::bottom(param) : sketch_policy(frac_mod_condition{fmh, param});
  std::vector<kmer_set> data = parallel_kmer_sets_from_fasta_files(n, files, mask, w, policy);
  std::vector<kmer_set> serial = kmer_sets_from_fasta_files(n, files, mask, w, policy);
  std::vector<kmer_set*> ptrs;
  for (auto& s : data) ptrs.push_back(&s);
  auto pairs = generate_all_pairs_from_vector<kmer_set*>(ptrs);
  (void)sks::take_pair_flow_stats();
  std::vector<int> inter = parallel_compute_pairwise_kmer_set_intersections(pairs.first, pairs.second);
  const sks::pair_flow_stats pst = sks::take_pair_flow_stats();
  std::vector<int> inter2 = compute_pairwise_kmer_set_intersections(pairs.first, pairs.second);

  std::printf("{\"mask\":\"%016llx%016llx\",\"k\":%d,\"sets\":[", (unsigned long long)mask.hi(),
              (unsigned long long)mask.lo(), kmer_num_indices);
  for (int i = 0; i < n; ++i) {
    if (i) std::printf(",");
    hexset(data[i]);
  }
  bool same = true;
  for (int i = 0; i < n; ++i) same = same && data[i].elements == serial[i].elements;
  std::printf("],\"serial_equal\":%s,\"devices\":%d,", same ? "true" : "false",
              (int)sks::parallel_devices().size());
  std::printf("\"pair_stats\":{\"calls\":%llu,\"devices\":%llu,\"h2d\":%llu,\"d2d\":%llu,\"d2h\":%llu},",
              (unsigned long long)pst.calls, (unsigned long long)pst.devices, (unsigned long long)pst.h2d_bytes,
              (unsigned long long)pst.d2d_bytes, (unsigned long long)pst.d2h_bytes);
  if (!same) {  // diagnostics: the serial build's sets
    std::printf("\"serial_sets\":[");
    for (int i = 0; i < n; ++i) {
      if (i) std::printf(",");
      hexset(serial[i]);
    }
    std::printf("],");
  }
  std::printf("\"inter\":[");
  for (size_t i = 0; i < inter.size(); ++i) std::printf("%s%d", i ? "," : "", inter[i]);
  std::printf("],\"inter_serial_equal\":%s,\"ani\":[", inter == inter2 ? "true" : "false");
  for (size_t i = 0; i < inter.size(); ++i) {
    double c = containment(inter[i], pairs.first[i]->kmer_set_size());
    std::printf("%s\"%a\"", i ? "," : "", binomial_estimator(c, kmer_num_indices));
  }
  // single-pair API and membership
  int single = n > 1 ? kmer_set_intersection(data[0], data[1]) : -1;
  std::printf("],\"single01\":%d", single);
  if (n > 0) {
    auto runs = nucleotide_strings_from_fasta_file(files[0]);
    kmer_set viaruns = nucleotide_string_list_to_kmer_set(runs, mask, w, policy);
    std::printf(",\"runs_equal\":%s", viaruns.elements == data[0].elements ? "true" : "false");
    auto raw = strings_from_fasta(files[0]);
    auto cut = cut_nucleotide_strings(raw);
    std::printf(",\"cut_equal\":%s,\"records\":%zu", cut == runs ? "true" : "false", raw.size());
  }
  std::printf("}\n");
  return 0;
}

static int errors() {
  int ok = 0;
  try {
    contiguous_kmer(65);
  } catch (const std::runtime_error& e) {
    ok += std::string(e.what()) == "Given k-mer length exceeds maximum k-mer length";
  }
  kmer_set a, b;
  std::vector<kmer_set*> one{&a}, two{&a, &b};
  try {
    compute_pairwise_kmer_set_intersections(one, two);
  } catch (const std::runtime_error& e) {
    ok += std::string(e.what()) ==
          "Lists of kmer sets for intersection computation have different lengths";
  }
  // canonical_kmer / reverse_complement on a palindromic contiguous mask (kmers.cpp)
  kmer_bitset m = contiguous_kmer(4);
  kmer x{4, kmer_bitset(0b00011011, 0), m, kmer_bitset(0b00011011, 0)};  // ACGT
  kmer rc = reverse_complement(x);
  ok += rc.masked_bits == kmer_bitset(0b00011011, 0);  // ACGT is its own reverse complement
  kmer y{4, kmer_bitset(0b11111111, 0), m, kmer_bitset(0b11111111, 0)};  // TTTT -> AAAA
  ok += canonical_kmer(y).masked_bits == kmer_bitset(0, 0);
  // insert_kmers collapses duplicates; contains()
  kmer_set s;
  s.insert_kmers({y, y, x});
  ok += s.kmer_set_size() == 2 && s.contains(x);
  // frac_min_hash matches sks_frac_min_hash
  frac_min_hash f(1);
  uint64_t kk[2] = {x.masked_bits.lo(), 0}, mm[2] = {m.lo(), 0};
  ok += f(x) == sks_frac_min_hash(kk, mm, 4, 1, 0);
  std::printf("{\"errors_ok\":%d}\n", ok);
  return ok == 6 ? 0 : 2;
}

// test_facade csv <out> <append 0|1> <w> <mask_lo hex> <mask_hi hex> <n> names1[n] names2[n] values[n]
static int csv(int argc, char** argv) {
  const std::string out = argv[2];
  const bool append = std::atoi(argv[3]) != 0;
  const int w = std::atoi(argv[4]);
  const kmer_bitset mask(std::strtoull(argv[5], nullptr, 16), std::strtoull(argv[6], nullptr, 16));
  const int n = std::atoi(argv[7]);
  if (argc != 8 + 3 * n) return 64;
  std::vector<std::string> a, b;
  std::vector<double> v;
  for (int i = 0; i < n; ++i) {
    a.emplace_back(argv[8 + i]);
    b.emplace_back(argv[8 + n + i]);
    v.push_back(std::strtod(argv[8 + 2 * n + i], nullptr));
  }
  write_to_csv(a, b, v, w, mask, out, append);
  return 0;
}

// test_facade list <w> <k> <mask_seed> <c> <file>: nucleotide_string_list_to_kmers
// on the file's runs; one line per kmer: kmer_bits masked_bits (hex)
static int list(char** argv) {
  const int w = std::atoi(argv[2]), k = std::atoi(argv[3]);
  const kmer_bitset mask = generate_random_spaced_seed_mask(w, k, std::strtoull(argv[4], nullptr, 10));
  const frac_mod_condition cond{frac_min_hash(1), std::strtoull(argv[5], nullptr, 10)};
  auto runs = nucleotide_strings_from_fasta_file(argv[6]);
  std::vector<kmer> ks = nucleotide_string_list_to_kmers(runs, mask, w, cond);
  for (const kmer& x : ks)
    std::printf("%llx%016llx %llx%016llx\n", (unsigned long long)x.kmer_bits.hi(),
                (unsigned long long)x.kmer_bits.lo(), (unsigned long long)x.masked_bits.hi(),
                (unsigned long long)x.masked_bits.lo());
  return 0;
}

// test_facade store <path> <window>: save three host sets, load them back;
// prints the elements (hex lo hi per line, sets separated by "--").
// test_facade load <path>: load and print the same way (errors -> exit 3).
static void print_sets(const std::vector<kmer_set>& sets, const std::vector<std::string>& names) {
  for (size_t i = 0; i < sets.size(); ++i) {
    std::printf("-- %s %d\n", names.empty() ? "" : names[i].c_str(), sets[i].window_length);
    for (const kmer_bitset& e : sets[i].elements)
      std::printf("%llx %llx\n", (unsigned long long)e.lo(), (unsigned long long)e.hi());
  }
}

static int store(char** argv) {
  const int w = std::atoi(argv[3]);
  const kmer_bitset mask = generate_random_spaced_seed_mask(w, w > 10 ? w - 5 : w, 0);
  std::vector<kmer_set> sets(3);
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < 3; ++i) {
    sets[i].window_length = w;
    sets[i].mask = mask;
    sets[i].has_mask = true;
    std::vector<kmer_bitset> v;
    for (int j = 0; j < 50 * i; ++j) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      v.push_back(kmer_bitset(x, 0) & mask);
    }
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    sets[i].elements = v;
  }
  sks::save_kmer_sets(argv[2], sets, sketch_policy::frac(200, 1), {"a.fa", "dir/b.fa", "c"});
  std::vector<std::string> names;
  sketch_policy pol;
  auto back = sks::load_kmer_sets(argv[2], &names, &pol);
  bool same = back.size() == sets.size() && pol.param == 200 && pol.kind == SKS_FRAC_MOD;
  for (size_t i = 0; same && i < sets.size(); ++i)
    same = back[i].elements == sets[i].elements && back[i].mask == mask;
  print_sets(back, names);
  return same ? 0 : 2;
}

// test_facade store_mixed <path> <case>: sets the reference's kmer_set can hold
// but one (window, mask) per file cannot — case 0: a set with k-mers under two
// masks (kmer.hpp:170-178), an empty set, a 40-wide set; case 1: one mask and
// an empty set among full ones (written as version 1).  Saves, loads, compares
// every field; prints "sets <n> sizes <size/other masks>..." (exit 2 on a
// mismatch).  A 5th argument "gpu" also compares all pair intersections.
static bool same_set(const kmer_set& a, const kmer_set& b) {
  if (a.has_mask != b.has_mask || a.elements != b.elements || a.kmer_set_size() != b.kmer_set_size())
    return false;
  if (a.has_mask && (a.mask != b.mask || a.window_length != b.window_length)) return false;
  if (a.other_masks.size() != b.other_masks.size()) return false;
  for (size_t g = 0; g < a.other_masks.size(); ++g)
    if (a.other_masks[g].mask != b.other_masks[g].mask ||
        a.other_masks[g].window_length != b.other_masks[g].window_length ||
        a.other_masks[g].elements != b.other_masks[g].elements)
      return false;
  return true;
}

static int store_mixed(char** argv) {
  const int which = std::atoi(argv[3]);
  const kmer_bitset m1 = generate_random_spaced_seed_mask(31, 21, 0);
  const kmer_bitset m2 = generate_random_spaced_seed_mask(31, 21, 5);
  const kmer_bitset m3 = generate_random_spaced_seed_mask(40, 30, 1);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  auto kmers = [&](const kmer_bitset& m, int w, int n) {
    std::vector<kmer> v;
    for (int j = 0; j < n; ++j) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      kmer_bitset bits(x, x * 31);
      v.push_back(kmer{w, bits, m, bits & m});
    }
    return v;
  };
  std::vector<kmer_set> sets(3);
  if (which == 0) {
    std::vector<kmer> a = kmers(m1, 31, 40), b = kmers(m2, 31, 25);
    a.insert(a.end(), b.begin(), b.end());
    a.push_back(a[3]);  // a duplicate collapses
    sets[0].insert_kmers(a);
    sets[2].insert_kmers(kmers(m3, 40, 30));
  } else {
    sets[0].insert_kmers(kmers(m1, 31, 40));
    sets[2].insert_kmers(kmers(m1, 31, 7));
  }
  sks::save_kmer_sets(argv[2], sets, sketch_policy::bottom(100, 1), {"mixed", "empty", "wide"});
  std::vector<std::string> names;
  sketch_policy pol;
  auto back = sks::load_kmer_sets(argv[2], &names, &pol);
  bool same = back.size() == sets.size() && pol.param == 100 && pol.kind == SKS_BOTTOM_S &&
              names == std::vector<std::string>{"mixed", "empty", "wide"};
  for (size_t i = 0; same && i < sets.size(); ++i) {
    if (which == 1 && sets[i].kmer_set_size() == 0) {
      // version 1 gives an empty set the file's mask; it stays empty
      same = back[i].kmer_set_size() == 0 && back[i].other_masks.empty();
      continue;
    }
    same = same_set(back[i], sets[i]);
  }
  // the loaded sets intersect like the originals (on the GPU: only with "gpu")
  const bool gpu = argv[4] && std::string(argv[4]) == "gpu";
  for (size_t i = 0; gpu && same && i < sets.size(); ++i)
    for (size_t j = 0; same && j < sets.size(); ++j)
      same = kmer_set_intersection(back[i], back[j]) == kmer_set_intersection(sets[i], sets[j]);
  std::printf("sets %zu sizes", back.size());
  for (const kmer_set& s : back) std::printf(" %d/%zu", s.kmer_set_size(), s.other_masks.size());
  std::printf("\n");
  return same ? 0 : 2;
}

static int load(char** argv) {
  try {
    std::vector<std::string> names;
    print_sets(sks::load_kmer_sets(argv[2], &names), names);
  } catch (const std::runtime_error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 3;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 64;
  std::string mode = argv[1];
  if (mode == "sketch" && argc >= 8) return sketch(argc, argv);
  if (mode == "errors") return errors();
  if (mode == "csv" && argc >= 8) return csv(argc, argv);
  if (mode == "list" && argc == 7) return list(argv);
  if (mode == "store" && argc == 4) return store(argv);
  if (mode == "load" && argc == 3) return load(argv);
  if (mode == "store_mixed" && (argc == 4 || argc == 5)) return store_mixed(argv);
  if (mode == "missing" && argc == 3) {
    char* f[1] = {argv[2]};
    kmer_bitset mask = generate_random_spaced_seed_mask(21, 21, 0);
    parallel_kmer_sets_from_fasta_files(1, f, mask, 21, frac_mod_condition{frac_min_hash(1), 200});
    return 0;  // unreachable: exit(1) like fasta_processing.cpp:86-90
  }
  return 64;
}
