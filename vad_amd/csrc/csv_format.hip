// Host-side text formatting of feature rows for the offline dataset export
// (reference dataset/file_processing.py:126-146 write_features through
// Python's csv writer, read back by load_csv :152-184 as float32).
//
// Each value is printed as numpy prints a float32 (str(np.float32(v))): the
// shortest digit string that round-trips, positional for 1e-4 <= |v| < 1e16
// (always with a fractional part, "3.0"), else scientific ("1e-05",
// "1.5e+16"); "nan", "inf", "-inf".  Fields are comma-separated and rows end
// in "\r\n" (the csv module's default dialect).  Row blocks are formatted on
// several host threads.
#include <charconv>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "vad_common.h"

namespace vad {

static char* fmt_f32(float v, char* p, char* end) {
  if (std::isnan(v)) {
    memcpy(p, "nan", 3);
    return p + 3;
  }
  if (std::isinf(v)) {
    if (v < 0) *p++ = '-';
    memcpy(p, "inf", 3);
    return p + 3;
  }
  const float a = std::fabs(v);
  if (a == 0.f) {
    if (std::signbit(v)) *p++ = '-';
    memcpy(p, "0.0", 3);
    return p + 3;
  }
  if ((double)a >= 1e16 || (double)a < 1e-4) {  // numpy decides on the exact value
    return std::to_chars(p, end, v, std::chars_format::scientific).ptr;
  }
  // positional: the shortest round-trip digits (from the scientific form),
  // zero-padded to the decimal point -- numpy prints 1.2573022e13 as
  // "12573022000000.0", not the exact binary value
  char sci[32];
  char* se = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific).ptr;
  const char* s = sci;
  if (*s == '-') {
    *p++ = '-';
    ++s;
  }
  char dig[24];
  int nd = 0;
  const char* ep = s;
  while (ep < se && *ep != 'e') {
    if (*ep != '.') dig[nd++] = *ep;
    ++ep;
  }
  int e = 0;
  std::from_chars(ep + 1 + (ep[1] == '+'), se, e);
  if (e >= 0) {
    for (int i = 0; i <= e; ++i) *p++ = i < nd ? dig[i] : '0';
    *p++ = '.';
    if (nd > e + 1) {
      for (int i = e + 1; i < nd; ++i) *p++ = dig[i];
    } else {
      *p++ = '0';
    }
  } else {
    *p++ = '0';
    *p++ = '.';
    for (int i = 0; i < -e - 1; ++i) *p++ = '0';
    for (int i = 0; i < nd; ++i) *p++ = dig[i];
  }
  (void)end;
  return p;
}

static char* fmt_label(double v, char* p, char* end) {
  // the label joins the float64 row (np.concatenate(..., [label])): small
  // integers print as "1.0"
  if (std::isfinite(v) && v == std::floor(v) && std::fabs(v) < 1e15) {
    char* q = std::to_chars(p, end, (long long)v).ptr;
    *q++ = '.';
    *q++ = '0';
    return q;
  }
  return std::to_chars(p, end, v).ptr;
}

static void format_block(const float* rows, int64_t r0, int64_t r1, int n_cols, double label,
                         std::string& out) {
  // worst case per value: sign + 9 significant digits + "e-45" ~ 16 chars
  out.resize((size_t)(r1 - r0) * ((size_t)n_cols * 24 + 48));
  char* p = out.data();
  char* end = p + out.size();
  for (int64_t r = r0; r < r1; ++r) {
    const float* x = rows + r * n_cols;
    for (int c = 0; c < n_cols; ++c) {
      p = fmt_f32(x[c], p, end);
      *p++ = ',';
    }
    p = fmt_label(label, p, end);
    *p++ = '\r';
    *p++ = '\n';
  }
  out.resize(p - out.data());
}

int64_t format_csv_rows(const float* rows, int64_t n_rows, int n_cols, double label, char* buf,
                        int64_t buf_size) {
  const int64_t per_thread = 8192;
  int n_threads = (int)((n_rows + per_thread - 1) / per_thread);
  const int hw = (int)std::thread::hardware_concurrency();
  const int cap = hw > 0 ? (hw < 16 ? hw : 16) : 4;
  if (n_threads > cap) n_threads = cap;
  if (n_threads < 1) n_threads = 1;
  std::vector<std::string> parts(n_threads);
  const int64_t chunk = (n_rows + n_threads - 1) / n_threads;
  if (n_threads == 1) {
    format_block(rows, 0, n_rows, n_cols, label, parts[0]);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) {
      const int64_t a = t * chunk, b = (t + 1) * chunk < n_rows ? (t + 1) * chunk : n_rows;
      th.emplace_back([=, &parts] { format_block(rows, a, b, n_cols, label, parts[t]); });
    }
    for (auto& t : th) t.join();
  }
  int64_t total = 0;
  for (auto& s : parts) total += (int64_t)s.size();
  if (!buf || total > buf_size) return -total;  // caller retries with a larger buffer
  char* p = buf;
  for (auto& s : parts) {
    memcpy(p, s.data(), s.size());
    p += s.size();
  }
  return total;
}

}  // namespace vad
