// ani_estimator.hpp — drop-in replacement for the reference's
// src/ani_estimator.hpp (ani_estimator.hpp:13-14); implemented by
// sks_containment / sks_binomial_estimator (bit-identical doubles).
#pragma once

#include <cmath>        // ani_estimator.hpp:11
#include "logging.hpp"  // ani_estimator.hpp:12

double containment(int intersection, int set_size);
double binomial_estimator(double containment, int kmer_num_ones);
