// Host-side helpers shared by the C-ABI translation units.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "sks.h"

// A device-resident set of sketches (one per genome / segment).
struct sks_sketch_set {
  int device = 0;
  int elem_words = 1;
  uint32_t n = 0;
  uint64_t* d_data = nullptr;    // elements (elem_words u64 each)
  uint64_t* d_starts = nullptr;  // [n] element index of each sketch
  uint32_t* d_sizes = nullptr;   // [n]
  std::vector<uint32_t> sizes;
  std::vector<uint64_t> starts;
  std::vector<uint64_t> windows;
  // how the sketches were made (persisted with them)
  int window = 0;
  uint64_t mask[2] = {0, 0};
  sks_policy policy{};
  std::vector<std::string> names;  // optional, from a sketch file or sks_sketch_set_set_name
};

namespace sks {

// Records `msg` as the calling thread's last error and returns `code`.
int fail(int code, const std::string& msg);

// fasta_processing.cpp:35-69: A/a->0 C/c->1 G/g->2 T/t->3, anything else 4.
inline uint8_t nucleotide_code(uint8_t ch) {
  switch (ch) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    case 't': case 'T': return 3;
    default: return 4;
  }
}

// ---- sketch files (persist.cpp) ----------------------------------------------------
struct SketchFileMeta {
  int window = 0;
  int elem_words = 1;
  uint64_t mask[2] = {0, 0};
  sks_policy policy{};
};
// Writes / reads the format documented in persist.cpp.  `data` holds the
// sketches back to back (sizes[i] * elem_words words each); names may be empty.
int write_sketch_file(const char* path, const SketchFileMeta& meta, const std::vector<uint32_t>& sizes,
                      const std::vector<uint64_t>& windows, const uint64_t* data,
                      const std::vector<std::string>& names);
int read_sketch_file(const char* path, SketchFileMeta& meta, std::vector<uint32_t>& sizes,
                     std::vector<uint64_t>& windows, std::vector<uint64_t>& data,
                     std::vector<std::string>& names);
// Version 2: sets made of (window, mask) groups (the facade's mixed-mask
// kmer_sets).  `data` holds the groups back to back, in set order.
struct SketchGroup {
  uint32_t set;
  int32_t window;
  uint64_t mask[2];
  uint64_t size;
};
int write_sketch_file_groups(const char* path, const SketchFileMeta& meta,
                             const std::vector<uint32_t>& sizes, const std::vector<uint64_t>& windows,
                             const std::vector<SketchGroup>& groups, const uint64_t* data,
                             const std::vector<std::string>& names);
// Reads version 1 or 2; `grouped` tells which (groups is empty for version 1).
int read_sketch_file_any(const char* path, SketchFileMeta& meta, std::vector<uint32_t>& sizes,
                         std::vector<uint64_t>& windows, std::vector<uint64_t>& data,
                         std::vector<std::string>& names, std::vector<SketchGroup>& groups,
                         bool& grouped);

void parse_fasta_bytes(const uint8_t* data, uint64_t n, sks_fasta* out);

}  // namespace sks
