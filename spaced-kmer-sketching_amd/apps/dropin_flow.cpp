// dropin-flow — the reference driver's sketching step exactly as an unmodified
// caller runs it (kmer-sketching.cpp:165-175): parallel_kmer_sets_from_fasta_files
// with the reference's global-function predicate sketching_condition (:29-34),
// passed as std::function<bool(const kmer)> — every window is extracted on the
// GPU and the predicate runs on the host — timed beside the same call with the
// device-side descriptor (sketch_policy::frac(200): selection on the GPU).
// Both must give the same sets.  Prints one JSON object per configuration.
//
//   dropin-flow <w:k,w:k,...> <a.fa> <b.fa> ...
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "kmer.hpp"

frac_min_hash fmh(1);
inline bool sketching_condition(const kmer& test_kmer) {  // kmer-sketching.cpp:29-34
  const int c = 200;
  return (fmh(test_kmer) % c == 0);
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char* argv[]) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <w:k,...> <fasta files...>\n", argv[0]);
    return 1;
  }
  std::vector<std::pair<int, int>> cfg;
  for (const char* q = argv[1]; *q;) {
    char* e = nullptr;
    const int w = (int)std::strtol(q, &e, 10);
    const int k = (int)std::strtol(e + 1, &e, 10);
    cfg.emplace_back(w, k);
    q = *e == ',' ? e + 1 : e;
  }
  const int n = argc - 2;
  char** files = argv + 2;
  try {
    {  // warm-up: the device workers (contexts, streams, pinned buffers) are created once per process
      const kmer_bitset m = generate_random_spaced_seed_mask(cfg[0].first, cfg[0].second);
      (void)parallel_kmer_sets_from_fasta_files(n, files, m, cfg[0].first, sketching_condition);
      (void)parallel_kmer_sets_from_fasta_files(n, files, m, cfg[0].first, sketch_policy::frac(200));
      (void)sks::take_window_flow_stats();
    }
    for (auto [w, k] : cfg) {
      const kmer_bitset mask = generate_random_spaced_seed_mask(w, k);
      auto t0 = std::chrono::steady_clock::now();
      std::vector<kmer_set> a = parallel_kmer_sets_from_fasta_files(n, files, mask, w, sketching_condition);
      const double fn_ms = ms_since(t0);
      const sks::window_flow_stats st = sks::take_window_flow_stats();
      t0 = std::chrono::steady_clock::now();
      std::vector<kmer_set> b = parallel_kmer_sets_from_fasta_files(n, files, mask, w, sketch_policy::frac(200));
      const double desc_ms = ms_since(t0);
      bool same = a.size() == b.size();
      uint64_t elems = 0;
      for (size_t i = 0; same && i < a.size(); ++i) {
        same = a[i].elements == b[i].elements;
        elems += a[i].elements.size();
      }
      std::printf("{\"w\": %d, \"k\": %d, \"files\": %d, \"threads\": %d, \"std_function_ms\": %.3f, "
                  "\"descriptor_ms\": %.3f, \"windows\": %llu, \"pieces\": %llu, \"d2h_bytes\": %llu, "
                  "\"d2h_ms_sum\": %.3f, \"wait_ms_sum\": %.3f, \"predicate_ms_sum\": %.3f, \"worker_ms_sum\": %.3f, "
                  "\"sketch_elements\": %llu, \"sets_equal\": %s}\n",
                  w, k, n, sks::host_threads(), fn_ms, desc_ms, (unsigned long long)st.windows,
                  (unsigned long long)st.pieces, (unsigned long long)st.d2h_bytes, st.d2h_ms, st.wait_ms,
                  st.predicate_ms, st.wall_ms, (unsigned long long)elems, same ? "true" : "false");
      std::fflush(stdout);
      if (!same) return 2;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "dropin-flow: %s\n", e.what());
    return 1;
  }
  return 0;
}
