// Thin extern "C" shim over the reference's OWN ingress and ANI sources,
// compiled (by oracle/Makefile) together with
//   /root/reference/src/fasta_processing.cpp
//   /root/reference/src/ani_estimation.cpp
// into oracle/_ref/libref_fasta_ani.so.  Test infrastructure only: it pins the
// oracle's restatement (oracle/sks_oracle.cpp) and generates tests/golden/.
// No reference source is copied; the headers are included from where they lie.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fasta_processing.hpp"
#include "ani_estimator.hpp"

extern "C" {
typedef struct {
  uint8_t* data;
  uint64_t* lens;
  uint64_t n;
  uint64_t total;
} refx_buf;
}

template <class V>
static void put(const std::vector<V>& v, refx_buf* out) {
  uint64_t total = 0;
  for (auto& s : v) total += s.size();
  out->n = v.size();
  out->total = total;
  out->data = (uint8_t*)malloc(total ? total : 1);
  out->lens = (uint64_t*)malloc(sizeof(uint64_t) * (v.size() ? v.size() : 1));
  uint64_t o = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    if (!v[i].empty()) memcpy(out->data + o, v[i].data(), v[i].size());
    o += v[i].size();
    out->lens[i] = v[i].size();
  }
}

extern "C" {

void refx_buf_free(refx_buf* b) {
  free(b->data);
  free(b->lens);
  b->data = nullptr;
  b->lens = nullptr;
}

// strings_from_fasta (exit(1)s on an unreadable file, like the reference).
void refx_fasta_records(const char* path, refx_buf* out) { put(strings_from_fasta(path), out); }

// nucleotide_strings_from_fasta_file.
void refx_fasta_runs(const char* path, refx_buf* out) {
  put(nucleotide_strings_from_fasta_file(path), out);
}

double refx_containment(int inter, int size) { return containment(inter, size); }
double refx_binomial_estimator(double c, int k) { return binomial_estimator(c, k); }

}  // extern "C"
