// Host-side persistence of kmer_sets on the SKSKETCH file format (persist.cpp).
//
// A collection where every non-empty set holds one group under one shared
// (window, mask) is written as version 1, the format the C ABI also reads.
// Anything else the reference's kmer_set can hold — k-mers under several masks
// in one set (kmer.hpp:170-178 inserts any mix), or sets under different masks —
// is written as version 2, one (window, mask) group per mask of each set, and
// loads back into the same elements / other_masks.
#include "sketch_io.hpp"

#include <stdexcept>

#include "sks_api_internal.hpp"

namespace sks {

namespace {

// Can the collection be written as version 1 (one window / mask for the file)?
// Returns the index of the set whose (window, mask) the file carries, or -1 if
// every set is empty (the file then carries `window` 1 and mask 0).
bool one_mask(const std::vector<kmer_set>& sets, int* carrier) {
  *carrier = -1;
  for (size_t i = 0; i < sets.size(); ++i) {
    const kmer_set& s = sets[i];
    if (!s.other_masks.empty()) return false;
    if (s.elements.empty()) continue;
    if (*carrier < 0) {
      *carrier = (int)i;
    } else if (s.window_length != sets[*carrier].window_length || s.mask != sets[*carrier].mask) {
      return false;
    }
  }
  return true;
}

void push_elements(std::vector<uint64_t>& data, const std::vector<kmer_bitset>& v, int words) {
  for (const kmer_bitset& e : v) {
    data.push_back(e.lo());
    if (words == 2) data.push_back(e.hi());
  }
}

}  // namespace

void save_kmer_sets(const std::string& path, const std::vector<kmer_set>& sets,
                    const sketch_policy& policy, const std::vector<std::string>& names) {
  SketchFileMeta meta;
  meta.policy = sks_policy{policy.kind, policy.flavour, policy.param, policy.nonce};
  std::vector<uint32_t> sizes;
  std::vector<uint64_t> windows(sets.size(), 0);  // not tracked by kmer_set: 0 = unknown
  std::vector<uint64_t> data;
  int carrier = -1;
  if (one_mask(sets, &carrier)) {
    meta.window = carrier < 0 ? 1 : sets[carrier].window_length;
    meta.elem_words = meta.window > 32 ? 2 : 1;
    if (carrier >= 0) {
      meta.mask[0] = sets[carrier].mask.lo();
      meta.mask[1] = sets[carrier].mask.hi();
    }
    for (const kmer_set& s : sets) {
      sizes.push_back((uint32_t)s.elements.size());
      push_elements(data, s.elements, meta.elem_words);
    }
    if (write_sketch_file(path.c_str(), meta, sizes, windows, data.data(), names) != SKS_OK)
      throw std::runtime_error(sks_last_error());
    return;
  }
  // version 2: each set as its list of (window, mask) groups
  std::vector<SketchGroup> groups;
  int wide = 1;
  for (const kmer_set& s : sets) {
    if (s.window_length > 32) wide = 2;
    for (const kmer_set::mask_group& g : s.other_masks)
      if (g.window_length > 32) wide = 2;
  }
  meta.elem_words = wide;
  for (uint32_t i = 0; i < sets.size(); ++i) {
    const kmer_set& s = sets[i];
    uint64_t n = 0;
    auto add = [&](int w, const kmer_bitset& m, const std::vector<kmer_bitset>& v) {
      if (w < 1 || w > 64) throw std::invalid_argument("save_kmer_sets: window length out of range");
      groups.push_back(SketchGroup{i, w, {m.lo(), m.hi()}, v.size()});
      push_elements(data, v, wide);
      n += v.size();
    };
    if (s.has_mask) add(s.window_length, s.mask, s.elements);
    for (const kmer_set::mask_group& g : s.other_masks) add(g.window_length, g.mask, g.elements);
    sizes.push_back((uint32_t)n);
  }
  meta.window = groups.front().window;  // not empty: one_mask failed, so some set has a group
  meta.mask[0] = groups.front().mask[0];
  meta.mask[1] = groups.front().mask[1];
  if (write_sketch_file_groups(path.c_str(), meta, sizes, windows, groups, data.data(), names) != SKS_OK)
    throw std::runtime_error(sks_last_error());
}

std::vector<kmer_set> load_kmer_sets(const std::string& path, std::vector<std::string>* names,
                                     sketch_policy* policy) {
  SketchFileMeta meta;
  std::vector<uint32_t> sizes;
  std::vector<uint64_t> windows, data;
  std::vector<std::string> nm;
  std::vector<SketchGroup> groups;
  bool grouped = false;
  if (read_sketch_file_any(path.c_str(), meta, sizes, windows, data, nm, groups, grouped) != SKS_OK)
    throw std::runtime_error(sks_last_error());
  const int ew = meta.elem_words;
  auto elem = [&](uint64_t e) {
    return ew == 1 ? kmer_bitset(data[e], 0) : kmer_bitset(data[2 * e], data[2 * e + 1]);
  };
  std::vector<kmer_set> out(sizes.size());
  uint64_t e = 0;
  if (!grouped) {
    const kmer_bitset mask(meta.mask[0], meta.mask[1]);
    for (size_t i = 0; i < sizes.size(); ++i) {
      kmer_set& ks = out[i];
      ks.window_length = meta.window;
      ks.mask = mask;
      ks.has_mask = true;
      ks.elements.reserve(sizes[i]);
      for (uint32_t j = 0; j < sizes[i]; ++j, ++e) ks.elements.push_back(elem(e));
    }
  } else {
    for (const SketchGroup& g : groups) {
      kmer_set& ks = out[g.set];
      std::vector<kmer_bitset> v;
      v.reserve(g.size);
      for (uint64_t j = 0; j < g.size; ++j, ++e) v.push_back(elem(e));
      const kmer_bitset m(g.mask[0], g.mask[1]);
      if (!ks.has_mask) {
        ks.window_length = g.window;
        ks.mask = m;
        ks.has_mask = true;
        ks.elements = std::move(v);
      } else {
        ks.other_masks.push_back(kmer_set::mask_group{g.window, m, std::move(v)});
      }
    }
  }
  if (names) *names = nm;
  if (policy) *policy = sketch_policy{meta.policy.kind, meta.policy.param, meta.policy.nonce, meta.policy.flavour};
  return out;
}

}  // namespace sks
