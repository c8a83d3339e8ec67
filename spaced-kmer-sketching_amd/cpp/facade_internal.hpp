// Helpers shared by the facade translation units (facade.cpp, sweep.cpp).
// Not part of the public API.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "sks.h"

namespace sks {

[[noreturn]] void raise(int rc);
void check(int rc);
void check_hip(hipError_t e, const char* what);
sks_ctx* ctx();  // the facade's context on the selected device (set_device)

// Device buffer owned by the facade (freed on destruction; not copyable), on
// `device` (-1: the facade's device, set_device).
struct DevMem {
  void* p = nullptr;
  int device = 0;
  size_t bytes = 0;
  explicit DevMem(size_t bytes, int device = -1);
  ~DevMem();
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Whole-file read; false if the file cannot be opened or read.
bool read_raw(const char* path, std::vector<uint8_t>& buf);
// The reference's unreadable-file behaviour (fasta_processing.cpp:86-90):
// stderr + exit(1), or an exception when set_exit_on_io_error(false).
void report_unreadable(const char* path);
// Reads files concurrently (the reference's cilk_for over files), reporting an
// unreadable one like the reference, in file order.
std::vector<std::vector<uint8_t>> read_files(int num_files, char* filenames[]);

}  // namespace sks
