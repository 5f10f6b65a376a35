// cg_parse.cpp -- the reference's cron spec grammar (node/cron/parser.go) on
// the host, with the same bitmask results and error texts.  Parsing stays on
// the CPU: it is per rule, tiny, and string-shaped.
#include "cg_parse.h"

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

namespace cg {

namespace {

struct Bounds {
  unsigned min, max;
  int names;  // 0 none, 1 months, 2 days of week
};
// spec.go:18-46
const Bounds kSeconds{0, 59, 0}, kMinutes{0, 59, 0}, kHours{0, 23, 0}, kDom{1, 31, 0},
    kMonths{1, 12, 1}, kDow{0, 6, 2};

const char* const kMonthNames[] = {"jan", "feb", "mar", "apr", "may", "jun",
                                   "jul", "aug", "sep", "oct", "nov", "dec"};
const char* const kDowNames[] = {"sun", "mon", "tue", "wed", "thu", "fri", "sat"};

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

std::string S(std::string_view v) { return std::string(v); }

// strconv.Quote for the characters a spec can carry
std::string quote(std::string_view s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      case '\r': o += "\\r"; break;
      case '\a': o += "\\a"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      case '\v': o += "\\v"; break;
      default:
        if (c < 0x20 || c == 0x7f) {
          static const char hx[] = "0123456789abcdef";
          o += "\\x";
          o += hx[c >> 4];
          o += hx[c & 15];
        } else {
          o += char(c);
        }
    }
  }
  return o + "\"";
}

// strconv.Atoi: 0 ok, 1 invalid syntax, 2 out of range
int atoi_go(std::string_view s, int64_t* out) {
  size_t n = s.size();
  if (n > 0 && n < 19) {  // fast path
    size_t i = 0;
    bool neg = false;
    if (s[0] == '-' || s[0] == '+') {
      neg = s[0] == '-';
      i = 1;
      if (n == 1) return 1;
    }
    int64_t v = 0;
    for (; i < n; i++) {
      unsigned d = unsigned(uint8_t(s[i]) - '0');
      if (d > 9) return 1;
      v = v * 10 + d;
    }
    *out = neg ? -v : v;
    return 0;
  }
  if (n == 0) return 1;  // ParseInt(s, 10, 0)
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i == n) return 1;
  uint64_t un = 0;
  bool range = false;
  for (; i < n; i++) {
    unsigned d = unsigned(uint8_t(s[i]) - '0');
    if (d > 9) return 1;
    if (range) continue;
    if (un > UINT64_MAX / 10 || un * 10 > UINT64_MAX - d) {
      range = true;
      continue;
    }
    un = un * 10 + d;
  }
  if (range) return 2;
  const uint64_t cutoff = 1ULL << 63;
  if ((!neg && un >= cutoff) || (neg && un > cutoff)) return 2;
  *out = neg ? int64_t(0 - un) : int64_t(un);
  return 0;
}

// mustParseInt, parser.go:280-290
bool must_parse_int(std::string_view s, uint64_t* out, std::string* err) {
  int64_t v = 0;
  int rc = atoi_go(s, &v);
  if (rc) {
    if (err)
      *err = fmt("Failed to parse int from %s: strconv.Atoi: parsing %s: %s", S(s).c_str(),
                 quote(s).c_str(), rc == 1 ? "invalid syntax" : "value out of range");
    return false;
  }
  if (v < 0) {
    if (err) *err = fmt("Negative number (%lld) not allowed: %s", (long long)v, S(s).c_str());
    return false;
  }
  *out = uint64_t(v);
  return true;
}

// parseIntOrName, parser.go:270-277
bool parse_int_or_name(std::string_view s, int names, uint64_t* out, std::string* err) {
  if (names && s.size() == 3) {
    char low[4] = {0, 0, 0, 0};
    for (int i = 0; i < 3; i++) {
      char c = s[i];
      low[i] = (c >= 'A' && c <= 'Z') ? char(c + 32) : c;
    }
    const char* const* tab = names == 1 ? kMonthNames : kDowNames;
    int cnt = names == 1 ? 12 : 7, base = names == 1 ? 1 : 0;
    for (int i = 0; i < cnt; i++)
      if (!std::strcmp(low, tab[i])) {
        *out = uint64_t(i + base);
        return true;
      }
  }
  return must_parse_int(s, out, err);
}

std::vector<std::string_view> split(std::string_view s, char sep) {
  std::vector<std::string_view> parts;
  size_t start = 0;
  for (size_t i = 0; i <= s.size(); i++) {
    if (i == s.size() || s[i] == sep) {
      parts.push_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  return parts;
}

// unicode.IsSpace on UTF-8 input: byte length of a space rune at s[i], or 0
size_t space_at(std::string_view s, size_t i) {
  auto b = [&](size_t k) { return i + k < s.size() ? uint8_t(s[i + k]) : 0u; };
  uint8_t c = b(0);
  if (c == ' ' || (c >= '\t' && c <= '\r')) return 1;
  if (c == 0xC2 && (b(1) == 0x85 || b(1) == 0xA0)) return 2;
  if (c == 0xE1 && b(1) == 0x9A && b(2) == 0x80) return 3;
  if (c == 0xE2 && b(1) == 0x80 &&
      ((b(2) >= 0x80 && b(2) <= 0x8A) || b(2) == 0xA8 || b(2) == 0xA9 || b(2) == 0xAF))
    return 3;
  if (c == 0xE2 && b(1) == 0x81 && b(2) == 0x9F) return 3;
  if (c == 0xE3 && b(1) == 0x80 && b(2) == 0x80) return 3;
  return 0;
}

std::vector<std::string_view> fields_of(std::string_view s) {  // strings.Fields
  std::vector<std::string_view> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t sp = space_at(s, i);
    if (sp) {
      i += sp;
      continue;
    }
    size_t j = i;
    while (j < s.size() && !space_at(s, j)) j++;
    out.push_back(s.substr(i, j - i));
    i = j;
  }
  return out;
}

uint64_t all_bits(const Bounds& b) { return get_bits(b.min, b.max, 1) | kStarBit; }

int parse_descriptor(std::string_view d, Schedule* out, std::string* err) {
  // parser.go:314-377
  Schedule s;
  s.kind = 0;
  if (d == "@yearly" || d == "@annually") {
    s.second = 1; s.minute = 1; s.hour = 1; s.dom = 1ULL << 1; s.month = 1ULL << 1;
    s.dow = all_bits(kDow);
  } else if (d == "@monthly") {
    s.second = 1; s.minute = 1; s.hour = 1; s.dom = 1ULL << 1; s.month = all_bits(kMonths);
    s.dow = all_bits(kDow);
  } else if (d == "@weekly") {
    s.second = 1; s.minute = 1; s.hour = 1; s.dom = all_bits(kDom); s.month = all_bits(kMonths);
    s.dow = 1;
  } else if (d == "@daily" || d == "@midnight") {
    s.second = 1; s.minute = 1; s.hour = 1; s.dom = all_bits(kDom); s.month = all_bits(kMonths);
    s.dow = all_bits(kDow);
  } else if (d == "@hourly") {
    s.second = 1; s.minute = 1; s.hour = all_bits(kHours); s.dom = all_bits(kDom);
    s.month = all_bits(kMonths); s.dow = all_bits(kDow);
  } else if (d.size() >= 7 && d.substr(0, 7) == "@every ") {
    int64_t dur;
    std::string derr;
    if (parse_duration(d.substr(7), &dur, &derr)) {
      if (err) *err = fmt("Failed to parse duration %s: %s", S(d).c_str(), derr.c_str());
      return -1;
    }
    s.kind = 1;
    s.delay_ns = every(dur);
  } else {
    if (err) *err = fmt("Unrecognized descriptor: %s", S(d).c_str());
    return -1;
  }
  *out = s;
  return 0;
}

}  // namespace

uint64_t get_bits(unsigned min, unsigned max, unsigned step) {
  if (step == 1) {
    uint64_t hi = max + 1 >= 64 ? 0 : (~0ULL << (max + 1));
    uint64_t lo = min >= 64 ? 0 : (~0ULL << min);
    return ~hi & lo;
  }
  uint64_t bits = 0;
  for (uint64_t i = min; i <= max; i += step)
    if (i < 64) bits |= 1ULL << i;
  return bits;
}

int get_range(std::string_view expr, unsigned rmin, unsigned rmax, int names, uint64_t* bits,
              std::string* err) {
  // getRange, parser.go:204-267
  *bits = 0;
  auto range_and_step = split(expr, '/');
  auto low_and_high = split(range_and_step[0], '-');
  bool single = low_and_high.size() == 1;
  uint64_t start, end, step;
  uint64_t extra = 0;
  if (low_and_high[0] == "*" || low_and_high[0] == "?") {
    start = rmin;
    end = rmax;
    extra = kStarBit;
  } else {
    if (!parse_int_or_name(low_and_high[0], names, &start, err)) return -1;
    if (low_and_high.size() == 1) {
      end = start;
    } else if (low_and_high.size() == 2) {
      if (!parse_int_or_name(low_and_high[1], names, &end, err)) return -1;
    } else {
      if (err) *err = fmt("Too many hyphens: %s", S(expr).c_str());
      return -1;
    }
  }
  if (range_and_step.size() == 1) {
    step = 1;
  } else if (range_and_step.size() == 2) {
    if (!must_parse_int(range_and_step[1], &step, err)) return -1;
    if (single) end = rmax;  // "N/step" means "N-max/step"
  } else {
    if (err) *err = fmt("Too many slashes: %s", S(expr).c_str());
    return -1;
  }
  if (start < rmin) {
    if (err)
      *err = fmt("Beginning of range (%llu) below minimum (%u): %s", (unsigned long long)start,
                 rmin, S(expr).c_str());
    return -1;
  }
  if (end > rmax) {
    if (err)
      *err = fmt("End of range (%llu) above maximum (%u): %s", (unsigned long long)end, rmax,
                 S(expr).c_str());
    return -1;
  }
  if (start > end) {
    if (err)
      *err = fmt("Beginning of range (%llu) beyond end of range (%llu): %s",
                 (unsigned long long)start, (unsigned long long)end, S(expr).c_str());
    return -1;
  }
  if (step == 0) {
    if (err) *err = fmt("Step of range should be a positive number: %s", S(expr).c_str());
    return -1;
  }
  *bits = get_bits(unsigned(start), unsigned(end), step > 64 ? 64u : unsigned(step)) | extra;
  return 0;
}

int get_field(std::string_view field, unsigned min, unsigned max, int names, uint64_t* bits,
              std::string* err) {
  // getField, parser.go:188-199 (FieldsFunc drops empty pieces)
  uint64_t acc = 0;
  for (auto piece : split(field, ',')) {
    if (piece.empty()) continue;
    uint64_t b;
    if (get_range(piece, min, max, names, &b, err)) {
      *bits = acc;
      return -1;
    }
    acc |= b;
  }
  *bits = acc;
  return 0;
}

int64_t every(int64_t d) {
  // Every, constantdelay.go:14-21
  const int64_t sec = 1000000000LL;
  if (d < sec) d = sec;
  return d - d % sec;
}

int parse_duration(std::string_view s0, int64_t* out, std::string* err) {
  // time.ParseDuration
  static const struct {
    const char* u;
    uint64_t ns;
  } units[] = {{"ns", 1},
               {"us", 1000},
               {"\xC2\xB5s", 1000},
               {"\xCE\xBCs", 1000},
               {"ms", 1000000},
               {"s", 1000000000ULL},
               {"m", 60000000000ULL},
               {"h", 3600000000000ULL}};
  const uint64_t kTop = 1ULL << 63;
  std::string q = quote(s0);
  auto invalid = [&]() {
    if (err) *err = "time: invalid duration " + q;
    return -1;
  };
  std::string_view s = s0;
  uint64_t d = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
    neg = s[0] == '-';
    s.remove_prefix(1);
  }
  if (s == "0") {
    *out = 0;
    return 0;
  }
  if (s.empty()) return invalid();
  while (!s.empty()) {
    uint64_t v = 0, f = 0;
    double scale = 1;
    if (!(s[0] == '.' || (s[0] >= '0' && s[0] <= '9'))) return invalid();
    size_t pl = s.size();
    size_t i = 0;
    for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; i++) {  // leadingInt
      if (v > kTop / 10) return invalid();
      v = v * 10 + uint64_t(s[i] - '0');
      if (v > kTop) return invalid();
    }
    s.remove_prefix(i);
    bool pre = pl != s.size();
    bool post = false;
    if (!s.empty() && s[0] == '.') {
      s.remove_prefix(1);
      size_t pl2 = s.size();
      bool overflow = false;
      size_t k = 0;
      for (; k < s.size() && s[k] >= '0' && s[k] <= '9'; k++) {  // leadingFraction
        if (overflow) continue;
        if (f > (kTop - 1) / 10) {
          overflow = true;
          continue;
        }
        uint64_t y = f * 10 + uint64_t(s[k] - '0');
        if (y > kTop) {
          overflow = true;
          continue;
        }
        f = y;
        scale *= 10;
      }
      s.remove_prefix(k);
      post = pl2 != s.size();
    }
    if (!pre && !post) return invalid();
    size_t u = 0;
    while (u < s.size() && !(s[u] == '.' || (s[u] >= '0' && s[u] <= '9'))) u++;
    if (u == 0) {
      if (err) *err = "time: missing unit in duration " + q;
      return -1;
    }
    std::string_view us = s.substr(0, u);
    s.remove_prefix(u);
    uint64_t unit = 0;
    for (auto& e : units)
      if (us == e.u) unit = e.ns;
    if (!unit) {
      if (err) *err = "time: unknown unit " + quote(us) + " in duration " + q;
      return -1;
    }
    if (v > kTop / unit) return invalid();
    v *= unit;
    if (f > 0) {
      v += uint64_t(double(f) * (double(unit) / scale));
      if (v > kTop) return invalid();
    }
    d += v;
    if (d > kTop) return invalid();
  }
  if (neg) {
    *out = int64_t(0 - d);
    return 0;
  }
  if (d > kTop - 1) return invalid();
  *out = int64_t(d);
  return 0;
}

int parse(int options, std::string_view spec, Schedule* out, std::string* err) {
  // NewParser, parser.go:66-73
  int optionals = 0;
  if (options & OPT_DOW_OPTIONAL) {
    options |= OPT_DOW;
    optionals++;
  }
  *out = Schedule();
  if (spec.empty()) {
    if (err) *err = "runtime error: index out of range [0] with length 0";
    return -2;
  }
  if (spec[0] == '@' && (options & OPT_DESCRIPTOR)) return parse_descriptor(spec, out, err);

  static const int places[6] = {OPT_SECOND, OPT_MINUTE, OPT_HOUR, OPT_DOM, OPT_MONTH, OPT_DOW};
  static const char* const defaults[6] = {"0", "0", "0", "*", "*", "*"};
  int max = 0;
  for (int p : places)
    if (options & p) max++;
  int min = max - optionals;
  auto fields = fields_of(spec);
  int count = int(fields.size());
  if (count < min || count > max) {
    if (err) {
      if (min == max)
        *err = fmt("Expected exactly %d fields, found %d: %s", min, count, S(spec).c_str());
      else
        *err = fmt("Expected %d to %d fields, found %d: %s", min, max, count, S(spec).c_str());
    }
    return -1;
  }
  std::string_view ex[6];
  for (int i = 0; i < 6; i++) ex[i] = defaults[i];
  int n = 0;  // expandFields, parser.go:138-153
  for (int i = 0; i < 6; i++) {
    if (options & places[i]) {
      if (n >= count) {  // Go indexes fields[n] and panics
        if (err) *err = fmt("runtime error: index out of range [%d] with length %d", n, count);
        return -2;
      }
      ex[i] = fields[n++];
    }
    if (n == count) break;
  }
  const Bounds* b[6] = {&kSeconds, &kMinutes, &kHours, &kDom, &kMonths, &kDow};
  uint64_t v[6];
  for (int i = 0; i < 6; i++)
    if (get_field(ex[i], b[i]->min, b[i]->max, b[i]->names, &v[i], err)) return -1;
  out->kind = 0;
  out->second = v[0];
  out->minute = v[1];
  out->hour = v[2];
  out->dom = v[3];
  out->month = v[4];
  out->dow = v[5];
  return 0;
}

}  // namespace cg

// ------------------------------------------------- C-ABI: parse (host) ---
// cg_parse*, cg_get_*, cg_every, cg_parse_duration (include/cronsun_gpu.h);
// host-only, so the sanitizer build (tests/test_sanitizers.py) covers them.
#include <algorithm>
#include <thread>

#include "../../include/cronsun_gpu.h"

int cg_fail(int code, const std::string& msg);

using namespace cg;

extern "C" {

static void fill_schedule(const Schedule& s, cg_schedule* out) {
  std::memset(out, 0, sizeof *out);
  out->kind = s.kind;
  out->second = s.second;
  out->minute = s.minute;
  out->hour = s.hour;
  out->dom = s.dom;
  out->month = s.month;
  out->dow = s.dow;
  out->delay_ns = s.delay_ns;
}

int cg_parse(int options, const char* spec, size_t len, cg_schedule* out, char* err,
             size_t err_cap) {
  if (!out || (!spec && len)) return cg_fail(CG_EINVAL, "cg_parse: null argument");
  Schedule s;
  std::string e;
  int rc = parse(options, std::string_view(spec ? spec : "", len), &s, &e);
  if (rc != 0) {
    if (err && err_cap) {
      std::strncpy(err, e.c_str(), err_cap - 1);
      err[err_cap - 1] = 0;
    }
    return cg_fail(rc == -2 ? CG_EPANIC : CG_EPARSE, e);
  }
  fill_schedule(s, out);
  return CG_OK;
}

int cg_parse_batch(int options, const char* const* specs, const size_t* lens, size_t n,
                   cg_schedule* out, int32_t* status, int nthreads) {
  if (n && (!specs || !lens || !out || !status)) return cg_fail(CG_EINVAL, "cg_parse_batch: null");
  if (nthreads < 1) nthreads = 1;
  if (size_t(nthreads) > n / 1024 + 1) nthreads = int(n / 1024 + 1);
  auto work = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) {
      Schedule s;
      std::string e;
      int rc = parse(options, std::string_view(specs[i] ? specs[i] : "", lens[i]), &s, &e);
      if (rc == 0) {
        fill_schedule(s, &out[i]);
        status[i] = CG_OK;
      } else {
        std::memset(&out[i], 0, sizeof out[i]);
        status[i] = rc == -2 ? CG_EPANIC : CG_EPARSE;
      }
    }
  };
  std::vector<std::thread> th;
  size_t chunk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    size_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo >= hi) break;
    th.emplace_back(work, lo, hi);
  }
  for (auto& x : th) x.join();
  return CG_OK;
}

static int range_common(bool field, const char* expr, size_t len, unsigned min, unsigned max,
                        int names, uint64_t* bits, char* err, size_t err_cap) {
  if (!bits || (!expr && len)) return cg_fail(CG_EINVAL, "cg_get_range: null");
  std::string e;
  std::string_view v(expr ? expr : "", len);
  int rc = field ? get_field(v, min, max, names, bits, &e) : get_range(v, min, max, names, bits, &e);
  if (rc) {
    if (err && err_cap) {
      std::strncpy(err, e.c_str(), err_cap - 1);
      err[err_cap - 1] = 0;
    }
    return cg_fail(CG_EPARSE, e);
  }
  return CG_OK;
}

int cg_get_range(const char* expr, size_t len, unsigned min, unsigned max, int names,
                 uint64_t* bits, char* err, size_t err_cap) {
  return range_common(false, expr, len, min, max, names, bits, err, err_cap);
}

int cg_get_field(const char* expr, size_t len, unsigned min, unsigned max, int names,
                 uint64_t* bits, char* err, size_t err_cap) {
  return range_common(true, expr, len, min, max, names, bits, err, err_cap);
}

uint64_t cg_get_bits(unsigned min, unsigned max, unsigned step) { return get_bits(min, max, step); }

int64_t cg_every(int64_t d) { return every(d); }

int cg_parse_duration(const char* s, size_t len, int64_t* out) {
  if (!out) return cg_fail(CG_EINVAL, "cg_parse_duration: null");
  std::string e;
  if (parse_duration(std::string_view(s ? s : "", len), out, &e)) return cg_fail(CG_EPARSE, e);
  return CG_OK;
}

}  // extern "C"
