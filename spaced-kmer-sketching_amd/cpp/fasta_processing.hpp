// fasta_processing.hpp — drop-in replacement for the reference's
// src/fasta_processing.hpp (fasta_processing.hpp:18-23), backed by libsks.so's
// host ingress (sks_fasta_*).  Same record rules, same run cutting, and the
// same exit(1) on an unreadable file (see sks::set_exit_on_io_error).
#pragma once

#include <cstdint>
#include <fstream>   // fasta_processing.hpp:14-15
#include <iostream>
#include <string>
#include <vector>

#include "logging.hpp"  // fasta_processing.hpp:16

typedef std::vector<uint8_t> acgt_string;

std::vector<std::string> strings_from_fasta(const char fasta_filename[]);
void add_nucleotide_strings(std::vector<acgt_string>& return_strings, const std::string& raw_string);
std::vector<acgt_string> cut_nucleotide_strings(const std::vector<std::string>& raw_strings);
std::vector<acgt_string> nucleotide_strings_from_fasta_file(const char fasta_filename[]);
