// genome_batch, the CSV writer and the per-configuration ANI step of the
// reference driver (src/kmer-sketching.cpp:46-212) on libsks.so.
#include "sweep.hpp"

#include <chrono>
#include <fstream>
#include <iostream>
#include <memory>

#include "ani_estimator.hpp"
#include "facade_internal.hpp"
#include "generators.hpp"

void write_to_csv(const std::vector<std::string>& filenames1,
                  const std::vector<std::string>& filenames2,
                  const std::vector<double>& estimated_values, const int window_size,
                  const kmer_bitset& mask, const std::string& output_filename, bool is_append) {
  std::ofstream out(output_filename, is_append ? std::ios_base::out | std::ios_base::app
                                               : std::ios_base::out);
  if (!out.is_open()) {
    std::cerr << "Error: Unable to open file " << output_filename << " for writing." << std::endl;
    return;
  }
  if (!is_append) out << "File 1,File 2,Estimated Value,Window Size,Mask" << std::endl;
  const size_t rows = std::min({filenames1.size(), filenames2.size(), estimated_values.size()});
  const std::string mask_text = mask.to_string();
  for (size_t r = 0; r < rows; ++r)
    out << filenames1[r] << ',' << filenames2[r] << ',' << estimated_values[r] << ','
        << window_size << ',' << mask_text << std::endl;
}

namespace sks {

struct genome_batch::impl {
  std::vector<std::string> names;
  std::unique_ptr<DevMem> stream;  // record streams of all files, back to back
  std::vector<uint64_t> off;       // file i = stream[off[i], off[i+1])
  // the all-pairs step's buffers, kept across configurations (a hipFree per
  // configuration synchronises the device): the n x n count tiles and two
  // status words on the device, the n x n ANI matrix in pinned host memory
  // mapped into the device (the join writes it)
  std::unique_ptr<DevMem> counts, status;
  double* ani_host = nullptr;
  std::unique_ptr<std::pair<std::vector<std::string>, std::vector<std::string>>> names_pairs[2];
  ~impl() {
    if (ani_host) sks_host_free(ani_host);
  }
};

genome_batch::genome_batch(int num_files, char* filenames[]) : p_(new impl) {
  const int n = num_files > 0 ? num_files : 0;
  for (int i = 0; i < n; ++i) p_->names.emplace_back(filenames[i]);
  std::vector<std::vector<uint8_t>> raws = read_files(n, filenames);
  std::vector<uint64_t> in_off(1, 0);
  for (auto& r : raws) in_off.push_back(in_off.back() + r.size());
  DevMem d_raw(in_off.back());
  for (int i = 0; i < n; ++i)
    if (!raws[i].empty())
      check_hip(hipMemcpy(d_raw.as<uint8_t>() + in_off[i], raws[i].data(), raws[i].size(),
                          hipMemcpyHostToDevice), "hipMemcpy H2D");
  raws.clear();
  p_->stream.reset(new DevMem(in_off.back() + n));  // a stream is at most raw + 1 bytes
  p_->off.assign(1, 0);
  for (int i = 0; i < n; ++i) {
    uint64_t nb = 0, nr = 0;
    const uint64_t len = in_off[i + 1] - in_off[i];
    check(sks_fasta_parse_device(ctx(), d_raw.as<uint8_t>() + in_off[i], len,
                                 p_->stream->as<uint8_t>() + p_->off.back(), len + 1, nullptr, 0,
                                 &nb, &nr));
    p_->off.push_back(p_->off.back() + nb);
  }
  check(sks_ctx_synchronize(ctx()));
}

genome_batch::~genome_batch() { delete p_; }

size_t genome_batch::size() const { return p_->names.size(); }
const std::vector<std::string>& genome_batch::filenames() const { return p_->names; }

const std::pair<std::vector<std::string>, std::vector<std::string>>& genome_batch::pair_names(
    pair_mode mode) const {
  auto& slot = p_->names_pairs[mode == pair_mode::all_pairs ? 0 : 1];
  if (!slot)
    slot.reset(new std::pair<std::vector<std::string>, std::vector<std::string>>(
        mode == pair_mode::all_pairs ? generate_all_pairs_from_vector(p_->names)
                                     : generate_pairwise_from_vector(p_->names)));
  return *slot;
}
uint64_t genome_batch::stream_bytes() const { return p_->off.back(); }

namespace {
double ms_since(std::chrono::high_resolution_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t0)
      .count();
}
}  // namespace

genome_batch::comparison genome_batch::compare(const kmer_bitset& mask, int window_size,
                                               const sketch_policy& policy, pair_mode mode,
                                               int kmer_num_ones) const {
  comparison res;
  const uint32_t n = (uint32_t)size();
  if (n == 0) return res;
  auto t0 = std::chrono::high_resolution_clock::now();
  sks_policy pol{policy.kind, policy.flavour, policy.param, policy.nonce};
  const uint64_t m[2] = {mask.lo(), mask.hi()};
  sks_sketch_set* set = nullptr;
  check(sks_sketch_build(ctx(), p_->stream->as<uint8_t>(), p_->off.back(), p_->off.data(), n,
                         window_size, m, &pol, &set));
  std::unique_ptr<sks_sketch_set, int (*)(sks_sketch_set*)> guard(set, sks_sketch_set_free);
  std::vector<uint32_t> sizes(n);
  check(sks_sketch_set_sizes(set, sizes.data()));
  res.sketch_ms = ms_since(t0);

  t0 = std::chrono::high_resolution_clock::now();
  const uint64_t* data = sks_sketch_set_device_data(set);
  const uint64_t* starts = sks_sketch_set_device_starts(set);
  const uint32_t* dsizes = sks_sketch_set_device_sizes(set);
  const int ew = sks_sketch_set_elem_words(set);
  if (mode == pair_mode::all_pairs && kmer_num_ones > 0 && n <= 16384) {
    // kmer-sketching.cpp:185-200 in one native call: the join layout of the n
    // sketches, every upper-triangle 64 x 64 tile in one k_join launch, and
    // containment / ANI of both orientations written by each tile's last
    // workgroup straight into the pinned host matrix (no count read-back, no
    // host pow loop)
    const uint64_t pairs = (uint64_t)n * n, tiles = sks_intersect_sym_tiles(n);
    uint64_t total = 0;
    uint32_t max_size = 1;
    for (uint32_t v : sizes) {
      total += v;
      max_size = std::max(max_size, v);
    }
    if (!p_->counts || p_->counts->bytes < tiles * 4096 * 4) p_->counts.reset(new DevMem(tiles * 4096 * 4));
    if (!p_->status) p_->status.reset(new DevMem(8));
    if (!p_->ani_host) {
      void* h = nullptr;
      check(sks_host_alloc(pairs * sizeof(double), 0, &h));
      p_->ani_host = static_cast<double*>(h);
    }
    check(sks_all_pairs_ani(ctx(), data, starts, dsizes, ew, n, max_size, std::max<uint64_t>(total, 1),
                            kmer_num_ones, p_->ani_host, p_->counts->as<int32_t>(),
                            p_->status->as<uint32_t>()));
    check(sks_ctx_synchronize(ctx()));
    uint32_t stat[2] = {0, 0};
    check_hip(hipMemcpy(stat, p_->status->p, 8, hipMemcpyDeviceToHost), "D2H");
    if (stat[1] == 0) {
      res.ani.assign(p_->ani_host, p_->ani_host + pairs);
      res.compare_ms = ms_since(t0);
      return res;
    }
    // a layout that could not place a value group (adversarial 128-bit
    // values): count with sks_intersect_all below, ANI on the host
  }
  if (mode == pair_mode::all_pairs) {
    const uint64_t pairs = (uint64_t)n * n;
    DevMem d_out(pairs * 4);
    check(sks_intersect_all(ctx(), data, starts, dsizes, ew, n, 0, n, d_out.as<int32_t>()));
    res.intersections.resize(pairs);
    check(sks_ctx_synchronize(ctx()));
    check_hip(hipMemcpy(res.intersections.data(), d_out.p, pairs * 4, hipMemcpyDeviceToHost), "D2H");
    res.first_sizes.resize(pairs);
    for (uint64_t i = 0; i < n; ++i)
      for (uint64_t j = 0; j < n; ++j) res.first_sizes[i * n + j] = (int)sizes[i];
  } else {
    std::vector<int32_t> a(n), b(n);
    for (uint32_t i = 0; i < n; ++i) {
      a[i] = (int32_t)i;
      b[i] = (int32_t)((i + 1) % n);
    }
    DevMem d_a(n * 4), d_b(n * 4), d_out(n * 4);
    check_hip(hipMemcpy(d_a.p, a.data(), n * 4, hipMemcpyHostToDevice), "H2D");
    check_hip(hipMemcpy(d_b.p, b.data(), n * 4, hipMemcpyHostToDevice), "H2D");
    check(sks_intersect_pairs(ctx(), data, starts, dsizes, ew, d_a.as<int32_t>(), d_b.as<int32_t>(),
                              n, d_out.as<int32_t>()));
    check(sks_ctx_synchronize(ctx()));
    res.intersections.resize(n);
    check_hip(hipMemcpy(res.intersections.data(), d_out.p, n * 4, hipMemcpyDeviceToHost), "D2H");
    res.first_sizes.assign(sizes.begin(), sizes.end());
  }
  res.compare_ms = ms_since(t0);
  return res;
}

void ani_sweep_config(const genome_batch& batch, pair_mode mode, int window_size, int kmer_size,
                      const std::string& output_filename, bool is_append, std::ostream& log,
                      const sketch_policy& policy) {
  const kmer_bitset mask = generate_random_spaced_seed_mask(window_size, kmer_size);
  const int kmer_num_indices = (int)(mask.count() / NUCLEOTIDE_BIT_SIZE);
  genome_batch::comparison c = batch.compare(mask, window_size, policy, mode, kmer_num_indices);
  log << "Time taken for sketching = " << c.sketch_ms << " ms" << std::endl;
  auto t0 = std::chrono::high_resolution_clock::now();
  std::vector<double> ani = std::move(c.ani);
  if (ani.empty()) {  // the counts came back instead (adjacent pairs, or the fallback)
    ani.resize(c.intersections.size());
    for (size_t i = 0; i < ani.size(); ++i)
      ani[i] = binomial_estimator(containment(c.intersections[i], c.first_sizes[i]), kmer_num_indices);
  }
  const auto& names = batch.pair_names(mode);
  log << "Time taken for comparison = " << c.compare_ms + ms_since(t0) << " ms" << std::endl;
  write_to_csv(names.first, names.second, ani, window_size, mask, output_filename, is_append);
}

std::vector<std::pair<int, int>> reference_sweep_configs() {
  std::vector<std::pair<int, int>> cfg{{10, 10}};
  for (int k = 11; k <= 40; ++k) cfg.emplace_back(k, k);
  for (int k = 10; k <= 40; ++k) cfg.emplace_back(k + 10, k);
  return cfg;
}

}  // namespace sks
