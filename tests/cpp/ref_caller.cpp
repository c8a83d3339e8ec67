// A caller written against the reference's own API only (kmer.hpp,
// ani_estimator.hpp, fasta_processing.hpp, generators.hpp names and
// signatures): the experiment of kmer-sketching.cpp:151-212 — mask, sketch all
// files with a std::function predicate, all ordered pairs, intersections,
// containment and ANI — with the reference's global-function predicate
// (kmer-sketching.cpp:29-34) and with lambdas.  Nothing here names libsks.
// Prints JSON for tests/test_facade.py.
//   ref_caller <w> <k> <c> <file>...
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "ani_estimator.hpp"
#include "fasta_processing.hpp"
#include "generators.hpp"
#include "kmer.hpp"

static frac_min_hash fmh(1);
static unsigned long long g_c = 200;

// the reference's predicate shape: a free function taking the kmer by value
bool sketching_condition(const kmer k) { return fmh(k) % g_c == 0; }

static void print_hex(const kmer_bitset& b, bool comma) {
  std::printf("%s\"%016llx%016llx\"", comma ? "," : "", (unsigned long long)b.hi(),
              (unsigned long long)b.lo());
}

static void print_set(const kmer_set& ks) {
  // through the reference's member: kmer_hashes (unordered, so sort the keys)
  std::vector<kmer_bitset> keys;
  for (auto& [km, one] : ks.kmer_hashes)
    if (one == 1) keys.push_back(km.masked_bits);
  std::sort(keys.begin(), keys.end());
  std::printf("[");
  for (size_t i = 0; i < keys.size(); ++i) print_hex(keys[i], i > 0);
  std::printf("]");
}

template <typename set_pairs_fn, typename name_pairs_fn>
static void ani_experiment(set_pairs_fn make_set_pairs, name_pairs_fn make_name_pairs, int window_size,
                           int kmer_size, int num_files, char* filenames[]) {
  kmer_bitset mask = generate_random_spaced_seed_mask(window_size, kmer_size);
  const int kmer_num_indices = mask.count() / NUCLEOTIDE_BIT_SIZE;

  std::vector<kmer_set> data =
      parallel_kmer_sets_from_fasta_files(num_files, filenames, mask, window_size, sketching_condition);
  std::vector<kmer_set*> set_ptrs;
  std::vector<std::string> names;
  for (int i = 0; i < (int)data.size(); ++i) {
    set_ptrs.push_back(&data[i]);
    names.push_back(std::string(filenames[i]));
  }
  auto set_pairs = make_set_pairs(set_ptrs);
  auto name_pairs = make_name_pairs(names);
  std::vector<int> inter = parallel_compute_pairwise_kmer_set_intersections(set_pairs.first, set_pairs.second);
  std::vector<double> cont(inter.size()), ani(inter.size());
  for (size_t i = 0; i < inter.size(); ++i) {
    cont[i] = containment(inter[i], set_pairs.first[i]->kmer_set_size());
    ani[i] = binomial_estimator(cont[i], kmer_num_indices);
  }

  std::printf("{\"mask\":\"%016llx%016llx\",\"k\":%d,\"sets\":[", (unsigned long long)mask.hi(),
              (unsigned long long)mask.lo(), kmer_num_indices);
  for (size_t i = 0; i < data.size(); ++i) {
    if (i) std::printf(",");
    print_set(data[i]);
  }
  std::printf("],\"pairs\":[");
  for (size_t i = 0; i < name_pairs.first.size(); ++i)
    std::printf("%s[\"%s\",\"%s\"]", i ? "," : "", name_pairs.first[i].c_str(), name_pairs.second[i].c_str());
  std::printf("],\"inter\":[");
  for (size_t i = 0; i < inter.size(); ++i) std::printf("%s%d", i ? "," : "", inter[i]);
  std::printf("],\"ani\":[");
  for (size_t i = 0; i < ani.size(); ++i) std::printf("%s\"%a\"", i ? "," : "", ani[i]);
  std::printf("]");

  // serial builders with a lambda (same predicate), and a stateful lambda
  // counting its calls: once per window, like kmer_sliding.cpp:183
  std::vector<kmer_set> serial = kmer_sets_from_fasta_files(
      num_files, filenames, mask, window_size, [](const kmer k) { return fmh(k) % g_c == 0; });
  bool same = serial.size() == data.size();
  for (size_t i = 0; same && i < data.size(); ++i)
    same = serial[i].kmer_set_size() == data[i].kmer_set_size() &&
           serial[i].kmer_hashes.size() == data[i].kmer_hashes.size();
  for (size_t i = 0; same && i < data.size(); ++i)
    for (auto& kv : data[i].kmer_hashes) same = same && serial[i].kmer_hashes.count(kv.first) == 1;
  std::printf(",\"lambda_equal\":%s", same ? "true" : "false");
  std::atomic<unsigned long long> calls{0};
  kmer_set one = kmer_set_from_fasta_file(filenames[0], mask, window_size, [&calls](const kmer k) {
    ++calls;
    return fmh(k) % g_c == 0;
  });
  std::printf(",\"calls0\":%llu,\"one_size\":%d", calls.load(), one.kmer_set_size());

  // a predicate no sketch descriptor expresses: keep masked k-mers whose
  // low word has an even number of set bits and is 1 mod 3 on its low 32 bits
  auto odd_rule = [](const kmer k) {
    const unsigned long long lo = k.masked_bits.lo();
    return (__builtin_popcountll(lo) % 2 == 0) && ((lo & 0xffffffffull) % 3 == 1);
  };
  kmer_set custom = kmer_set_from_fasta_file(filenames[0], mask, window_size, odd_rule);
  std::printf(",\"custom\":");
  print_set(custom);

  // the list API on the runs, same custom rule: every selected window in order
  std::vector<acgt_string> runs = nucleotide_strings_from_fasta_file(filenames[0]);
  std::vector<kmer> listed = nucleotide_string_list_to_kmers(runs, mask, window_size, odd_rule);
  std::printf(",\"list\":[");
  for (size_t i = 0; i < listed.size(); ++i) {
    std::printf("%s[", i ? "," : "");
    print_hex(listed[i].kmer_bits, false);
    print_hex(listed[i].masked_bits, true);
    std::printf("]");
  }
  std::printf("]");

  // k-mers of two masks in one set (identity is (masked_bits, mask), kmer.hpp:82-85)
  if (num_files > 1) {
    kmer_bitset mask2 = generate_random_spaced_seed_mask(window_size, kmer_size, 5);
    std::vector<kmer_set> mixed(2);
    for (int f = 0; f < 2; ++f) {
      std::vector<acgt_string> r = nucleotide_strings_from_fasta_file(filenames[f]);
      mixed[f].insert_kmers(nucleotide_string_list_to_kmers(r, mask, window_size, sketching_condition));
      mixed[f].insert_kmers(nucleotide_string_list_to_kmers(r, mask2, window_size, sketching_condition));
    }
    std::printf(",\"mask2\":\"%016llx%016llx\",\"mixed_sizes\":[%d,%d],\"mixed_inter\":%d",
                (unsigned long long)mask2.hi(), (unsigned long long)mask2.lo(), mixed[0].kmer_set_size(),
                mixed[1].kmer_set_size(), kmer_set_intersection(mixed[0], mixed[1]));
    std::vector<kmer_set*> p1{&mixed[0], &mixed[1], &mixed[0]}, p2{&mixed[1], &data[1], &mixed[0]};
    std::vector<int> mi = compute_pairwise_kmer_set_intersections(p1, p2);
    std::printf(",\"mixed_pairs\":[%d,%d,%d]", mi[0], mi[1], mi[2]);
  }
  std::printf("}\n");
}

int main(int argc, char* argv[]) {
  if (argc < 5) return 64;
  initialise_contiguous_kmer_array();
  initialise_reversing_kmer_array();
  const int w = std::atoi(argv[1]), k = std::atoi(argv[2]);
  g_c = std::strtoull(argv[3], nullptr, 10);
  ani_experiment(
      [](const std::vector<kmer_set*>& v) { return generate_all_pairs_from_vector(v); },
      [](const std::vector<std::string>& v) { return generate_all_pairs_from_vector(v); }, w, k,
      argc - 4, argv + 4);
  return 0;
}
