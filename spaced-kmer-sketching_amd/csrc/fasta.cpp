// FASTA ingress (host) — the reference's record rules from
// fasta_processing.cpp:79-133 (strings_from_fasta) and run cutting from
// :144-198, re-implemented as a single pass over the file bytes.
//
// Output is the device-ready "record stream": each record's content followed
// by one '\n' separator.  The stream is what sks_sketch_build consumes; a
// non-ACGT byte ends a run there exactly as it does in the reference.
//
// Record rules (getline semantics, '\n'-separated lines, '\r' kept):
//   * a line that is empty or starts with '>' closes the current record
//     (pushed if a name is set — even when empty) and, if non-empty, sets the
//     name to the rest of the line; the content restarts empty;
//   * lines before any header, or after a header with an empty name, are
//     ignored;
//   * a sequence line containing ' ' drops the record so far and clears the
//     name (so following lines are ignored until the next header);
//   * otherwise the line is appended to the content.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sks.h"
#include "sks_api_internal.hpp"

struct sks_fasta {
  std::vector<uint8_t> stream;    // record bytes, each record followed by '\n'
  std::vector<uint64_t> rec_off;  // record i = stream[rec_off[i], rec_off[i+1] - 1)
};

namespace {

bool read_file(const char* path, std::vector<uint8_t>& buf) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  buf.clear();
  if (fseek(f, 0, SEEK_END) == 0) {
    long n = ftell(f);
    if (n > 0) buf.reserve((size_t)n);
    fseek(f, 0, SEEK_SET);
  }
  uint8_t tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
  bool ok = !ferror(f);
  fclose(f);
  return ok;
}

}  // namespace

namespace sks {

void parse_fasta_bytes(const uint8_t* data, uint64_t n, sks_fasta* out) {
  std::vector<uint8_t>& s = out->stream;
  std::vector<uint64_t>& off = out->rec_off;
  s.clear();
  off.clear();
  s.reserve(n + 16);
  bool have_name = false;
  uint64_t cur = 0;  // start of the current record's content in s
  auto push = [&]() {
    off.push_back(cur);
    s.push_back('\n');
    cur = s.size();
  };
  uint64_t pos = 0;
  while (pos < n) {
    const uint8_t* nl = (const uint8_t*)memchr(data + pos, '\n', n - pos);
    uint64_t end = nl ? (uint64_t)(nl - data) : n;
    const uint8_t* line = data + pos;
    uint64_t len = end - pos;
    pos = nl ? end + 1 : n;
    if (len == 0 || line[0] == '>') {
      if (have_name) push();
      if (len != 0) have_name = len > 1;
      s.resize(cur);  // content.clear()
    } else if (have_name) {
      if (memchr(line, ' ', len) != nullptr) {
        have_name = false;
        s.resize(cur);
      } else {
        s.insert(s.end(), line, line + len);
      }
    }
  }
  if (have_name) push();
  s.resize(cur);  // drop an unterminated dropped record's content
  off.push_back(s.size());
}

}  // namespace sks

extern "C" {

int sks_fasta_open(const char* path, sks_fasta** out) {
  if (!path || !out) return sks::fail(SKS_E_ARG, "sks_fasta_open: null argument");
  *out = nullptr;
  std::vector<uint8_t> buf;
  if (!read_file(path, buf))
    return sks::fail(SKS_E_IO, std::string("Unable to open ") + path + ". \n Exiting...");
  sks_fasta* f = new (std::nothrow) sks_fasta();
  if (!f) return sks::fail(SKS_E_NOMEM, "sks_fasta_open: out of memory");
  sks::parse_fasta_bytes(buf.data(), buf.size(), f);
  *out = f;
  return SKS_OK;
}

void sks_fasta_close(sks_fasta* f) { delete f; }

uint64_t sks_fasta_num_records(const sks_fasta* f) { return f ? f->rec_off.size() - 1 : 0; }

int sks_fasta_record(const sks_fasta* f, uint64_t i, const uint8_t** data, uint64_t* len) {
  if (!f || !data || !len) return sks::fail(SKS_E_ARG, "sks_fasta_record: null argument");
  if (i + 1 >= f->rec_off.size()) return sks::fail(SKS_E_ARG, "sks_fasta_record: index out of range");
  *data = f->stream.data() + f->rec_off[i];
  *len = f->rec_off[i + 1] - f->rec_off[i] - 1;
  return SKS_OK;
}

const uint8_t* sks_fasta_stream(const sks_fasta* f) { return f ? f->stream.data() : nullptr; }

uint64_t sks_fasta_stream_bytes(const sks_fasta* f) { return f ? f->stream.size() : 0; }

int sks_fasta_runs(const sks_fasta* f, uint8_t* codes, uint64_t* run_lens, uint64_t* n_codes,
                   uint64_t* n_runs) {
  if (!f || !n_codes || !n_runs) return sks::fail(SKS_E_ARG, "sks_fasta_runs: null argument");
  const bool fill = codes && run_lens;
  const uint64_t cap_codes = *n_codes, cap_runs = *n_runs;
  uint64_t nc = 0, nr = 0, cur = 0;
  for (uint8_t ch : f->stream) {
    uint8_t b = sks::nucleotide_code(ch);
    if (b & 4) {
      if (cur) {
        if (fill && nr < cap_runs) run_lens[nr] = cur;
        ++nr;
      }
      cur = 0;
    } else {
      if (fill && nc < cap_codes) codes[nc] = b;
      ++nc;
      ++cur;
    }
  }
  if (cur) {  // unreachable: the stream always ends with a separator
    if (fill && nr < cap_runs) run_lens[nr] = cur;
    ++nr;
  }
  *n_codes = nc;
  *n_runs = nr;
  if (fill && (nc > cap_codes || nr > cap_runs))
    return sks::fail(SKS_E_ARG, "sks_fasta_runs: buffers too small");
  return SKS_OK;
}

}  // extern "C"
