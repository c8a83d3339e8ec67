// Host-side persistence of kmer_sets on the SKSKETCH file format (persist.cpp).
#include "sketch_io.hpp"

#include <stdexcept>

#include "sks_api_internal.hpp"

namespace sks {

void save_kmer_sets(const std::string& path, const std::vector<kmer_set>& sets,
                    const sketch_policy& policy, const std::vector<std::string>& names) {
  SketchFileMeta meta;
  meta.window = sets.empty() ? 1 : sets[0].window_length;
  meta.elem_words = meta.window > 32 ? 2 : 1;
  if (!sets.empty()) {
    meta.mask[0] = sets[0].mask.lo();
    meta.mask[1] = sets[0].mask.hi();
  }
  meta.policy = sks_policy{policy.kind, policy.flavour, policy.param, policy.nonce};
  std::vector<uint32_t> sizes;
  std::vector<uint64_t> windows(sets.size(), 0);  // not tracked by kmer_set: 0 = unknown
  std::vector<uint64_t> data;
  for (const kmer_set& s : sets) {
    if (s.window_length != meta.window || s.mask != sets[0].mask)
      throw std::runtime_error("save_kmer_sets: sets differ in window length or mask");
    sizes.push_back((uint32_t)s.elements.size());
    for (const kmer_bitset& e : s.elements) {
      data.push_back(e.lo());
      if (meta.elem_words == 2) data.push_back(e.hi());
    }
  }
  if (write_sketch_file(path.c_str(), meta, sizes, windows, data.data(), names) != SKS_OK)
    throw std::runtime_error(sks_last_error());
}

std::vector<kmer_set> load_kmer_sets(const std::string& path, std::vector<std::string>* names,
                                     sketch_policy* policy) {
  SketchFileMeta meta;
  std::vector<uint32_t> sizes;
  std::vector<uint64_t> windows, data;
  std::vector<std::string> nm;
  if (read_sketch_file(path.c_str(), meta, sizes, windows, data, nm) != SKS_OK)
    throw std::runtime_error(sks_last_error());
  std::vector<kmer_set> out(sizes.size());
  const kmer_bitset mask(meta.mask[0], meta.mask[1]);
  uint64_t e = 0;
  for (size_t i = 0; i < sizes.size(); ++i) {
    kmer_set& ks = out[i];
    ks.window_length = meta.window;
    ks.mask = mask;
    ks.has_mask = true;
    ks.elements.reserve(sizes[i]);
    for (uint32_t j = 0; j < sizes[i]; ++j, ++e)
      ks.elements.push_back(meta.elem_words == 1 ? kmer_bitset(data[e], 0)
                                                 : kmer_bitset(data[2 * e], data[2 * e + 1]));
  }
  if (names) *names = nm;
  if (policy) *policy = sketch_policy{meta.policy.kind, meta.policy.param, meta.policy.nonce, meta.policy.flavour};
  return out;
}

}  // namespace sks
