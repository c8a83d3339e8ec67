// generators.hpp — the reference's pair generators (generators.hpp:20-58):
// adjacent ring pairs and all ordered pairs including (i, i), i-major.
#pragma once

#include <cstddef>
#include <utility>
#include <vector>

#include "stl_includes.hpp"  // generators.hpp:10

template <typename T>
std::pair<std::vector<T>, std::vector<T>> generate_pairwise_from_vector(const std::vector<T>& v) {
  std::vector<T> first, second;
  const std::size_t n = v.size();
  first.reserve(n);
  second.reserve(n);
  for (std::size_t i = 0; i < n; ++i) {
    first.push_back(v[i]);
    second.push_back(v[(i + 1) % n]);
  }
  return {std::move(first), std::move(second)};
}

template <typename T>
std::pair<std::vector<T>, std::vector<T>> generate_all_pairs_from_vector(const std::vector<T>& v) {
  std::vector<T> first, second;
  const std::size_t n = v.size();
  first.reserve(n * n);
  second.reserve(n * n);
  for (std::size_t i = 0; i < n; ++i)
    for (std::size_t j = 0; j < n; ++j) {
      first.push_back(v[i]);
      second.push_back(v[j]);
    }
  return {std::move(first), std::move(second)};
}
