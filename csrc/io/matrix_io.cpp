// Parallel text/binary matrix reader (mmap, two passes, one copy) + writer + corner printer
// (see gj/io.hpp).
#include <fcntl.h>
#include <locale.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstdint>
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

inline bool is_ws(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// strtod in the C locale on a NUL-terminated copy of [b, e) (the mapping has no terminator).
const char* strtod_c(const char* b, const char* e, double& v) {
  static locale_t cloc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
  char small[128];
  std::string big;
  const size_t len = (size_t)(e - b);
  char* s = small;
  if (len + 1 > sizeof small) {
    big.assign(b, len);
    s = &big[0];
  } else {
    std::memcpy(small, b, len);
    small[len] = '\0';
  }
  char* endp = nullptr;
  v = strtod_l(s, &endp, cloc);
  return b + (endp - s);
}

// One whitespace-delimited token as scanf("%lf") would read it: 1 = exactly one number that
// consumes the token, 0 = not a number (the scan stops here), -1 = irregular (a number followed
// by more characters: scanf would go on inside the token, e.g. "1.5-3" is two numbers).
// Fast path std::from_chars (locale-free); hex floats, overflow and anything unusual go through
// strtod in the C locale, which has scanf's accept set.
int parse_token(const char* b, const char* e, double& v) {
  const char* s = b;
  bool neg = false;
  if (s < e && (*s == '+' || *s == '-')) neg = (*s++ == '-');
  const bool hex = (e - s >= 2 && s[0] == '0' && (s[1] == 'x' || s[1] == 'X'));
  if (!hex && s < e && *s != '+' && *s != '-') {
    const auto r = std::from_chars(s, e, v, std::chars_format::general);
    if (r.ec == std::errc() && r.ptr == e) {
      if (neg) v = -v;
      return 1;
    }
  }
  const char* q = strtod_c(b, e, v);
  if (q == b) return 0;
  return q == e ? 1 : -1;
}

// Lexical test: the token is one plain decimal number ([sign] digits[.digits] [e[sign]digits]) that
// strtod consumes completely.  Every other token (hex, inf/nan, glued numbers, garbage) is
// "suspect" and gets the full parse_token, also in rows this rank does not keep: scanf's result for
// the rows it keeps depends on every token before them (a glued "1.5-3" is two values, "zz" ends
// the read), so every rank must see the same irregularities, not only the row's owner.
inline bool plain_number(const char* b, const char* e) {
  const char* s = b;
  if (s < e && (*s == '+' || *s == '-')) ++s;
  int digits = 0;
  while (s < e && *s >= '0' && *s <= '9') ++s, ++digits;
  if (s < e && *s == '.') {
    ++s;
    while (s < e && *s >= '0' && *s <= '9') ++s, ++digits;
  }
  if (digits == 0) return false;
  if (s < e && (*s == 'e' || *s == 'E')) {
    ++s;
    if (s < e && (*s == '+' || *s == '-')) ++s;
    int ed = 0;
    while (s < e && *s >= '0' && *s <= '9') ++s, ++ed;
    if (ed == 0) return false;
  }
  return s == e;
}

struct Mapping {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  ~Mapping() {
    if (p && n) munmap(const_cast<char*>(p), n);
    if (fd >= 0) close(fd);
  }
};

// Give the pages of [b, e) of a read-only file mapping back (the page cache keeps them): the
// reader's resident set stays at its output plus a window per thread.
void drop_pages(const Mapping& mp, const char* b, const char* e) {
  const size_t pg = 4096;
  uintptr_t lo = ((uintptr_t)b + pg - 1) & ~(uintptr_t)(pg - 1);
  const uintptr_t hi = (uintptr_t)e & ~(uintptr_t)(pg - 1);
  (void)mp;
  if (hi > lo) madvise((void*)lo, hi - lo, MADV_DONTNEED);
}

// Exact sequential scanf("%lf") loop (fallback for irregular files): values [0, need) of the
// selected rows (rowpos[r] >= 0) into out.
Status scan_sequential(const Mapping& mp, size_t need, int64_t ncols, const std::vector<int64_t>& rowpos,
                       std::vector<double>& out) {
  const char* p = mp.p;
  const char* e = mp.p + mp.n;
  size_t idx = 0;
  while (idx < need) {
    while (p < e && is_ws(*p)) ++p;
    if (p >= e) return Status::CannotRead;
    const char* t = p;
    while (t < e && !is_ws(*t)) ++t;
    double v;
    const char* q = strtod_c(p, t, v);
    if (q == p) return Status::CannotRead;
    const int64_t r = (int64_t)(idx / (size_t)ncols), c = (int64_t)(idx % (size_t)ncols);
    if (rowpos[r] >= 0) out[(size_t)rowpos[r] * ncols + c] = v;
    ++idx;
    p = q;
  }
  return Status::Ok;
}

// The reader: the first nrows * ncols numbers of a text file (scanf("%lf") accept set) or raw fp64
// ".bin", keeping the rows with rowpos[r] >= 0 at output row rowpos[r].  Text: the file is mapped;
// pass 1 counts the tokens of every thread's chunk (chunks cut at whitespace), so every thread
// knows the global index of its first token; pass 2 parses only the selected tokens straight into
// the final buffer (no intermediate copies); the tokens of rows it does not keep get only the
// lexical plain_number test.  An irregular token (two numbers glued together) anywhere among the
// first nrows * ncols makes the whole read fall back to the exact sequential scan, on every rank.
Status read_rows(const std::string& path, int64_t nrows, int64_t ncols, const std::vector<int64_t>& rowpos,
                 int64_t nsel, std::vector<double>& out, int nthreads) {
  const size_t need = (size_t)nrows * (size_t)ncols;
  out.assign((size_t)nsel * (size_t)ncols, 0.0);
  Mapping mp;
  mp.fd = open(path.c_str(), O_RDONLY);
  if (mp.fd < 0) return Status::CannotOpen;
  struct stat sb;
  if (fstat(mp.fd, &sb) != 0) return Status::CannotRead;
  if (ends_with(path, ".bin")) {
    if ((size_t)sb.st_size < need * sizeof(double)) return Status::CannotRead;
    for (int64_t r = 0; r < nrows; ++r) {
      if (rowpos[r] < 0) continue;
      const size_t bytes = (size_t)ncols * sizeof(double);
      char* dst = reinterpret_cast<char*>(out.data() + (size_t)rowpos[r] * ncols);
      size_t got = 0;
      while (got < bytes) {
        const ssize_t k = pread(mp.fd, dst + got, bytes - got, (off_t)((size_t)r * bytes + got));
        if (k <= 0) return Status::CannotRead;
        got += (size_t)k;
      }
    }
    return Status::Ok;
  }
  mp.n = (size_t)sb.st_size;
  if (need == 0) return Status::Ok;
  if (mp.n == 0) return Status::CannotRead;
  void* a = mmap(nullptr, mp.n, PROT_READ, MAP_PRIVATE, mp.fd, 0);
  if (a == MAP_FAILED) return Status::CannotRead;
  mp.p = static_cast<const char*>(a);
  madvise(a, mp.n, MADV_SEQUENTIAL);
  const char* base = mp.p;
  const char* end = base + mp.n;

  int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  if (mp.n < (size_t)(1 << 20)) nt = 1;
  std::vector<const char*> cut(nt + 1);
  cut[0] = base;
  cut[nt] = end;
  for (int i = 1; i < nt; ++i) {
    const char* c = base + (mp.n * (size_t)i) / nt;
    if (c < cut[i - 1]) c = cut[i - 1];
    while (c < end && !is_ws(*c)) ++c;
    cut[i] = c;
  }
  const size_t kWindow = size_t(8) << 20;  // resident text per thread
  // pass 1: tokens per chunk
  std::vector<size_t> cnt(nt, 0);
  {
    std::vector<std::thread> th;
    for (int i = 0; i < nt; ++i)
      th.emplace_back([&, i] {
        size_t k = 0;
        bool in = false;
        const char* w0 = cut[i];
        for (const char* p = cut[i]; p < cut[i + 1]; ++p) {
          const bool ws = is_ws(*p);
          k += (!ws && !in);
          in = !ws;
          if ((size_t)(p - w0) >= kWindow) {
            drop_pages(mp, w0, p);
            w0 = p;
          }
        }
        drop_pages(mp, w0, cut[i + 1]);
        cnt[i] = k;
      });
    for (auto& t : th) t.join();
  }
  size_t total = 0;
  std::vector<size_t> first(nt);
  for (int i = 0; i < nt; ++i) {
    first[i] = total;
    total += cnt[i];
  }
  // fewer whitespace tokens than values: an error, unless glued tokens hold several numbers
  if (total < need) return scan_sequential(mp, need, ncols, rowpos, out);
  // pass 2: parse the selected tokens among the first `need`
  std::vector<int> err(nt, 0);  // 1 = invalid token inside [0, need), 2 = irregular token
  {
    std::vector<std::thread> th;
    for (int i = 0; i < nt; ++i)
      th.emplace_back([&, i] {
        size_t idx = first[i];
        if (idx >= need) return;
        const char* p = cut[i];
        const char* e = cut[i + 1];
        const char* w0 = p;
        while (idx < need) {
          while (p < e && is_ws(*p)) ++p;
          if (p >= e) break;
          const char* t = p;
          while (t < e && !is_ws(*t)) ++t;
          const int64_t r = (int64_t)(idx / (size_t)ncols);
          if (rowpos[r] < 0 && !plain_number(p, t)) {  // a row kept by another rank
            double v;
            const int ok = parse_token(p, t, v);
            if (ok == 0) {
              err[i] = 1;
              return;
            }
            if (ok < 0 && idx + 1 < need) {
              err[i] = 2;
              return;
            }
          }
          if (rowpos[r] >= 0) {
            double v;
            const int ok = parse_token(p, t, v);
            if (ok == 0) {
              err[i] = 1;
              return;
            }
            if (ok < 0) {  // the number prefix is value idx; what scanf does next is sequential
              err[i] = idx + 1 < need ? 2 : 0;
              out[(size_t)rowpos[r] * ncols + (int64_t)(idx % (size_t)ncols)] = v;
              if (err[i]) return;
            } else {
              out[(size_t)rowpos[r] * ncols + (int64_t)(idx % (size_t)ncols)] = v;
            }
          }
          ++idx;
          p = t;
          if ((size_t)(p - w0) >= kWindow) {
            drop_pages(mp, w0, p);
            w0 = p;
          }
        }
        drop_pages(mp, w0, p);
      });
    for (auto& t : th) t.join();
  }
  bool irregular = false;
  for (int i = 0; i < nt; ++i) {
    if (err[i] == 2) irregular = true;
    // an invalid token: an error unless an earlier chunk holds an irregular token (then the exact
    // sequential scan decides)
    if (err[i] == 1 && !irregular) return Status::CannotRead;
  }
  if (irregular) return scan_sequential(mp, need, ncols, rowpos, out);
  return Status::Ok;
}

}  // namespace

Status read_matrix_file(const std::string& path, int64_t n, std::vector<double>& out, int nthreads) {
  std::vector<int64_t> pos((size_t)n);
  for (int64_t r = 0; r < n; ++r) pos[r] = r;
  return read_rows(path, n, n, pos, n, out, nthreads);
}

Status read_matrix_rows(const std::string& path, int64_t n, const std::vector<int64_t>& rows,
                        std::vector<double>& out, int nthreads) {
  std::vector<int64_t> pos((size_t)n, -1);
  for (size_t i = 0; i < rows.size(); ++i) {
    GJ_REQUIRE(rows[i] >= 0 && rows[i] < n && pos[rows[i]] < 0, "read_matrix_rows: bad or repeated row");
    pos[rows[i]] = (int64_t)i;
  }
  return read_rows(path, n, n, pos, (int64_t)rows.size(), out, nthreads);
}

Status read_values_file(const std::string& path, size_t need, std::vector<double>& out, int nthreads) {
  std::vector<int64_t> pos(1, 0);
  return read_rows(path, 1, (int64_t)need, pos, 1, out, nthreads);
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
