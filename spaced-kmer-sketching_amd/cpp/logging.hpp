// logging.hpp — the reference's compile-time logging switches
// (src/logging.hpp:1-5), visible through kmer.hpp, fasta_processing.hpp and
// ani_estimator.hpp as in the reference.  Guarded the same way: a caller may
// define LOGGING (and with it INFO_LOG / DEBUG) before including any header.
#pragma once

#ifndef LOGGING
#define LOGGING 0
#define INFO_LOG "[INFO] "
#define DEBUG 0
#endif
