// sketch_io.hpp — persisted sketches for facade callers (no reference
// equivalent: the reference re-sketches every FASTA on every run).  Files use
// the "SKSKETCH" format of csrc/persist.cpp, shared with sks_sketch_set_save /
// sks_sketch_set_load, so sets saved from the C ABI load here and vice versa.
#pragma once

#include <string>
#include <vector>

#include "kmer.hpp"

namespace sks {

// Writes `sets` (all with the same window_length and mask) made with `policy`.
// `names` is empty or one name per set.  Host only; throws std::runtime_error.
void save_kmer_sets(const std::string& path, const std::vector<kmer_set>& sets,
                    const sketch_policy& policy, const std::vector<std::string>& names = {});

// Reads a sketch file into host kmer_sets; optionally returns names and policy.
std::vector<kmer_set> load_kmer_sets(const std::string& path, std::vector<std::string>* names = nullptr,
                                     sketch_policy* policy = nullptr);

}  // namespace sks
