// Host-side helpers shared by the C-ABI translation units.
#pragma once
#include <cstdint>
#include <string>

#include "sks.h"

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

void parse_fasta_bytes(const uint8_t* data, uint64_t n, sks_fasta* out);

}  // namespace sks
