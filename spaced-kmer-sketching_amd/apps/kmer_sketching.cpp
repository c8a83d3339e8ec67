// kmer-sketching — the reference's command-line driver (src/kmer-sketching.cpp:214-239)
// on the MI355X engine:
//
//   kmer-sketching <output.csv> <a.fa> <b.fa> ...
//
// Runs the reference's 62 (window, k) configurations over all ordered pairs of
// the given files and writes the same CSV (same rows, same bytes).  The files
// are read once and kept on the device (sks::genome_batch) instead of being
// re-parsed per configuration.  Extra option (not in the reference):
//   SKS_PAIRS=adjacent   ring pairs (i, i+1 mod n) instead of all pairs
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "sweep.hpp"

int main(int argc, char* argv[]) {
  if (argc < 2) {
    std::cerr << "usage: " << argv[0] << " <output.csv> <fasta files...>" << std::endl;
    return 1;
  }
  initialise_contiguous_kmer_array();
  initialise_reversing_kmer_array();
  const std::string output = argv[1];
  const char* pairs_env = std::getenv("SKS_PAIRS");
  const sks::pair_mode mode = pairs_env && std::strcmp(pairs_env, "adjacent") == 0
                                  ? sks::pair_mode::adjacent
                                  : sks::pair_mode::all_pairs;
  try {
    sks::genome_batch batch(argc - 2, argv + 2);
    bool append = false;
    for (auto [w, k] : sks::reference_sweep_configs()) {
      sks::ani_sweep_config(batch, mode, w, k, output, append, std::cout);
      append = true;
    }
  } catch (const std::exception& e) {
    std::cerr << "kmer-sketching: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
