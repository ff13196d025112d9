// Matrix file I/O and the reference-compatible stdout report.
//
// Reference: read_matrix (main.cpp:209-282; rank `sender` reads n*n numbers with fscanf("%lf"),
// errors -1 "cannot open" / -2 "cannot read"), print_row / print_matrix (main.cpp:284-341; the
// top-left min(n, MAX_P) square, "%.2f\t" per value).
#pragma once

#include <cstdio>
#include <string>
#include <vector>

#include "gj/common.hpp"

namespace gj {

// Reads the first n*n numbers of a whitespace-separated text file (row-major) with the same
// accept set as scanf("%lf").  Files ending in ".bin" are raw little-endian fp64 (n*n values).
// Returns Ok, CannotOpen or CannotRead.  Parsing is parallel (nthreads, 0 = auto).
Status read_matrix_file(const std::string& path, int64_t n, std::vector<double>& out, int nthreads = 0);
// Only the given rows (global row indices, each at most once) of the n x n matrix, in that order:
// out is rows.size() x n.  One rank's share in the one-process-per-GPU deployment: the file is
// mapped and every rank parses only its own rows (peak memory ~ its share + a window per thread);
// tokens of other rows are skipped, not validated (their owners validate them).
Status read_matrix_rows(const std::string& path, int64_t n, const std::vector<int64_t>& rows,
                        std::vector<double>& out, int nthreads = 0);
// Same parser for the first `count` numbers (right-hand sides: count = n).
Status read_values_file(const std::string& path, size_t count, std::vector<double>& out, int nthreads = 0);

// Writes an n x n fp64 matrix as text ("%.17g", one row per line) or raw binary (".bin").
Status write_matrix_file(const std::string& path, int64_t n, const double* a, int64_t ld);

// n values, one per line ("%.17g") or raw fp64 (".bin").
Status write_vector_file(const std::string& path, int64_t n, const double* x);

// print_row semantics: nm rows of nm values, "%.*f\t" each, newline per row.
void print_corner(FILE* f, const std::vector<double>& corner, int nm, int precision = 2);

}  // namespace gj
