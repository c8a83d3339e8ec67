// sweep.hpp — the reference driver's reusable pieces (src/kmer-sketching.cpp)
// for callers that evaluate many (window, k) configurations over one set of
// FASTA files: the CSV writer with the reference's exact output bytes, and a
// device-resident genome batch.
//
// The reference re-reads and re-parses every file for each of its 62
// configurations (kmer-sketching.cpp:168 inside the loops at :220-238).  A
// genome_batch reads the files once, parses them on the GPU
// (sks_fasta_parse_device) and keeps the record streams in HBM; each
// configuration then only re-sketches and re-intersects.
#pragma once

#include <ostream>
#include <string>
#include <vector>

#include "kmer.hpp"

// kmer-sketching.cpp:46-81.  Header "File 1,File 2,Estimated Value,Window Size,Mask"
// unless appending; one row per entry (min of the three lengths), values with
// the default ostream formatting, the mask as its 128-character bit string.
// An unopenable file prints the reference's message to stderr and returns.
void write_to_csv(const std::vector<std::string>& filenames1,
                  const std::vector<std::string>& filenames2,
                  const std::vector<double>& estimated_values, const int window_size,
                  const kmer_bitset& mask, const std::string& output_filename,
                  bool is_append = false);

namespace sks {

// generate_all_pairs_from_vector (i-major, including (i, i)) or
// generate_pairwise_from_vector (i, (i + 1) % n) — generators.hpp:20-58.
enum class pair_mode { all_pairs, adjacent };

class genome_batch {
 public:
  // Reads the files like parallel_kmer_sets_from_fasta_files (an unreadable
  // file exits like the reference) and parses them on the device.
  genome_batch(int num_files, char* filenames[]);
  ~genome_batch();
  genome_batch(const genome_batch&) = delete;
  genome_batch& operator=(const genome_batch&) = delete;

  size_t size() const;
  const std::vector<std::string>& filenames() const;
  // the file-name pairs of every configuration's CSV rows, generated once per
  // batch (the reference regenerates them per configuration, :180-183)
  const std::pair<std::vector<std::string>, std::vector<std::string>>& pair_names(pair_mode mode) const;
  uint64_t stream_bytes() const;

  struct comparison {
    std::vector<int> intersections;  // per pair, in generator order
    std::vector<int> first_sizes;    // kmer_set_size() of each pair's first set
    // all_pairs: binomial_estimator(containment(...)) of every pair, written by
    // the join itself (sks_all_pairs_ani, fp64 on the device; within 1e-9 of the
    // host's doubles); empty when the caller computes it from the counts
    std::vector<double> ani;
    double sketch_ms = 0, compare_ms = 0;  // host wall time of the two phases
  };
  // kmer_num_ones > 0 asks for the ANI with the counts (all_pairs mode).
  // Sketch every genome with (mask, window, policy), then count the pairs.
  comparison compare(const kmer_bitset& mask, int window_size, const sketch_policy& policy,
                     pair_mode mode, int kmer_num_ones = 0) const;

 private:
  struct impl;
  impl* p_;
};

// test_compute_ANI_estimation_random_spaced_kmers (kmer-sketching.cpp:151-212)
// on a resident batch: mask = generate_random_spaced_seed_mask(w, k), sketch
// with the reference's sketching_condition (frac_min_hash(1), c = 200), ANI =
// binomial_estimator(containment(inter, |first|), popcount(mask) / 2), timing
// lines to `log`, rows appended to the CSV exactly as the reference writes them.
void ani_sweep_config(const genome_batch& batch, pair_mode mode, int window_size, int kmer_size,
                      const std::string& output_filename, bool is_append, std::ostream& log,
                      const sketch_policy& policy = sketch_policy::frac(200, 1));

// The reference main's 62 (window, k) configurations, in order
// (kmer-sketching.cpp:218-238): (10,10); (k,k) k = 11..40; (k+10,k) k = 10..40.
std::vector<std::pair<int, int>> reference_sweep_configs();

}  // namespace sks
