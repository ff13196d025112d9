// Parallel text/binary matrix reader + writer + corner printer (see gj/io.hpp).
#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "gj/io.hpp"

namespace gj {

namespace {

bool ends_with(const std::string& s, const char* suf) {
  const size_t n = std::strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

// Parse numbers from [b, e) exactly like repeated scanf("%lf"): skip whitespace, strtod; a token
// strtod cannot convert stops the scan (error).  Returns count parsed; *err set when stopped early.
size_t parse_range(const char* b, const char* e, std::vector<double>& out, size_t limit, bool* err) {
  *err = false;
  const char* p = b;
  size_t cnt = 0;
  while (cnt < limit) {
    while (p < e && std::isspace((unsigned char)*p)) ++p;
    if (p >= e) break;
    char* endp = nullptr;
    errno = 0;
    const double v = std::strtod(p, &endp);
    if (endp == p) {
      *err = true;
      break;
    }
    out.push_back(v);
    ++cnt;
    p = endp;
  }
  return cnt;
}

}  // namespace

Status read_matrix_file(const std::string& path, int64_t n, std::vector<double>& out, int nthreads) {
  return read_values_file(path, (size_t)n * (size_t)n, out, nthreads);
}

Status read_values_file(const std::string& path, size_t need, std::vector<double>& out, int nthreads) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return Status::CannotOpen;
  if (ends_with(path, ".bin")) {
    out.assign(need, 0.0);
    const size_t got = std::fread(out.data(), sizeof(double), need, f);
    std::fclose(f);
    return got == need ? Status::Ok : Status::CannotRead;
  }
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (sz < 0) {
    std::fclose(f);
    return Status::CannotRead;
  }
  std::string buf((size_t)sz + 1, '\0');  // NUL-terminated so strtod never runs past the end
  const size_t rd = std::fread(&buf[0], 1, (size_t)sz, f);
  std::fclose(f);
  buf[rd] = '\0';
  const char* base = buf.data();
  const char* end = base + rd;

  int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  if (rd < (size_t)(1 << 20)) nt = 1;
  // chunk boundaries at whitespace
  std::vector<const char*> cut(nt + 1);
  cut[0] = base;
  cut[nt] = end;
  for (int i = 1; i < nt; ++i) {
    const char* c = base + (rd * (size_t)i) / nt;
    if (c < cut[i - 1]) c = cut[i - 1];
    while (c < end && !std::isspace((unsigned char)*c)) ++c;
    cut[i] = c;
  }
  std::vector<std::vector<double>> parts(nt);
  std::vector<char> errs(nt, 0);
  std::vector<std::thread> th;
  for (int i = 0; i < nt; ++i)
    th.emplace_back([&, i] {
      bool e = false;
      parts[i].reserve(need / nt + 16);
      parse_range(cut[i], cut[i + 1], parts[i], need, &e);
      errs[i] = e;
    });
  for (auto& t : th) t.join();
  out.clear();
  out.reserve(need);
  for (int i = 0; i < nt && out.size() < need; ++i) {
    const size_t take = std::min(parts[i].size(), need - out.size());
    out.insert(out.end(), parts[i].begin(), parts[i].begin() + take);
    if (errs[i] && out.size() < need) return Status::CannotRead;  // a bad token inside the first n*n
  }
  return out.size() == need ? Status::Ok : Status::CannotRead;
}

Status write_matrix_file(const std::string& path, int64_t n, const double* a, int64_t ld) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return Status::CannotOpen;
  if (ends_with(path, ".bin")) {
    for (int64_t i = 0; i < n; ++i) std::fwrite(a + i * ld, sizeof(double), (size_t)n, f);
  } else {
    for (int64_t i = 0; i < n; ++i) {
      for (int64_t j = 0; j < n; ++j) std::fprintf(f, j ? " %.17g" : "%.17g", a[i * ld + j]);
      std::fputc('\n', f);
    }
  }
  std::fclose(f);
  return Status::Ok;
}

Status write_vector_file(const std::string& path, int64_t n, const double* x) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return Status::CannotOpen;
  if (ends_with(path, ".bin"))
    std::fwrite(x, sizeof(double), (size_t)n, f);
  else
    for (int64_t i = 0; i < n; ++i) std::fprintf(f, "%.17g\n", x[i]);
  std::fclose(f);
  return Status::Ok;
}

void print_corner(FILE* f, const std::vector<double>& c, int nm, int precision) {
  for (int i = 0; i < nm; ++i) {
    for (int j = 0; j < nm; ++j) std::fprintf(f, "%.*f\t", precision, c[(size_t)i * nm + j]);
    std::fprintf(f, "\n");
  }
}

}  // namespace gj
