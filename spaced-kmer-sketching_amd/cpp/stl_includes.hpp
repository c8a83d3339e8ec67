// stl_includes.hpp — the standard-library surface the reference's headers make
// visible to their callers (src/stl_includes.hpp:15-31, pulled in by
// kmer.hpp:12 and generators.hpp:10).  Callers written against the reference
// (e.g. its kmer-sketching.cpp:24,56,64,166,175: std::cout, std::ofstream,
// std::cerr, std::chrono) rely on these transitively, so the facade keeps them.
// <numeric> is added because the facade's own callers often need std::iota,
// which the reference uses (kmer_bitset.cpp:140) without including it.
#pragma once

#include <algorithm>
#include <bitset>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <iterator>
#include <numeric>
#include <random>
#include <ranges>
#include <stdexcept>
#include <unordered_map>
#include <utility>
#include <vector>
