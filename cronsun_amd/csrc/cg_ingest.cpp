// cg_ingest.cpp -- bulk ingestion of cronsun's etcd values into a cg_jobset
// (SURVEY.md §8(f)-3).
//
// The reference loads every job with GetJobs (job.go:339-365): for each value
// under /cronsun/cmd/ it runs json.Unmarshal into Job (job.go:38-84; JobRule
// job.go:76-83), skips the value on any unmarshal error, skips it when
// Job.Valid fails (job.go:633-655: every rule's Timer through cron.Parse,
// JobRule.Valid job.go:291-308; the security checks are off unless
// configured), applies alone() (job.go:378-382), and keys the result by
// Job.ID (a later value with the same ID replaces an earlier one).  Groups
// come from GetGroups("") (group.go:39-63), keyed by Group.ID.
//
// The decoder restates Go 1.7/1.8 encoding/json (the reference's CI Go
// versions, .travis.yml) for exactly these two types:
//   * the whole value must be valid JSON (checkValid), else the value is
//     skipped; any type mismatch (UnmarshalTypeError) also skips it;
//   * object keys match field tags exactly, else ASCII case-insensitively
//     (non-letters exact; K U+212A and ſ U+017F fold to k and s for names that
//     contain k or s: fold.go); unknown keys are ignored; later duplicates win;
//   * null leaves a string/number/bool field unchanged and sets a slice or a
//     *JobRule to nil;
//   * arrays decode into the existing slice element by element (growing to
//     cap + cap/2, at least 4), reusing the elements already there -- so a
//     repeated "rules" key merges into the earlier *JobRule values -- and are
//     truncated to the array's length; an empty array leaves an empty slice;
//   * integers must parse with strconv.ParseInt (no fraction or exponent, in
//     int64 range);
//   * strings: escapes incl. \uXXXX surrogate pairs; lone surrogates and
//     invalid UTF-8 become U+FFFD.
// Documents are decoded on nthreads host threads; interning into the jobset
// is sequential.
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "cg_jobset.h"

namespace {

// ---- Go slice emulation: backing array of length cap, visible prefix len
template <class T>
struct GoSlice {
  std::vector<T> backing;
  size_t len = 0;
  bool nil = true;
  void set_nil() {
    backing.clear();
    len = 0;
    nil = true;
  }
};

struct PRule {
  std::string id, timer;
  GoSlice<std::string> gids, nids, ex;
};

struct PJob {
  std::string id, name, group, cmd, user;
  GoSlice<int32_t> rules;  // index into pool, -1 = nil pointer
  std::vector<PRule> pool;
  bool pause = false, fail_notify = false;
  int64_t timeout = 0, parallels = 0, retry = 0, interval = 0, kind = 0, avg_time = 0;
  GoSlice<std::string> to;
};

struct PGroup {
  std::string id, name;
  GoSlice<std::string> nids;
};

enum { kOk = 0, kSyntax = 1, kType = 2 };

struct Dec {
  const unsigned char* p;
  const unsigned char* e;
  int err = kOk;  // first error (syntax beats type: the whole value is validated first)

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
  }
  bool syntax() {
    err = kSyntax;
    return false;
  }
  void type_err() {
    if (err == kOk) err = kType;
  }
  bool lit(const char* s) {
    size_t n = std::strlen(s);
    if (size_t(e - p) < n || std::memcmp(p, s, n) != 0) return syntax();
    p += n;
    return true;
  }
  static void put_utf8(std::string* o, uint32_t r) {
    if (r < 0x80) {
      o->push_back(char(r));
    } else if (r < 0x800) {
      o->push_back(char(0xC0 | (r >> 6)));
      o->push_back(char(0x80 | (r & 0x3F)));
    } else if (r < 0x10000) {
      o->push_back(char(0xE0 | (r >> 12)));
      o->push_back(char(0x80 | ((r >> 6) & 0x3F)));
      o->push_back(char(0x80 | (r & 0x3F)));
    } else {
      o->push_back(char(0xF0 | (r >> 18)));
      o->push_back(char(0x80 | ((r >> 12) & 0x3F)));
      o->push_back(char(0x80 | ((r >> 6) & 0x3F)));
      o->push_back(char(0x80 | (r & 0x3F)));
    }
  }
  // one UTF-8 sequence at q (utf8.DecodeRune rules); returns length, r = rune
  // or 0xFFFD with length 1 when invalid
  static int decode_rune(const unsigned char* q, const unsigned char* end, uint32_t* r) {
    unsigned c = q[0];
    if (c < 0x80) { *r = c; return 1; }
    int n;
    uint32_t v, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) { n = 2; v = c & 0x1F; }
    else if (c >= 0xE0 && c <= 0xEF) {
      n = 3; v = c & 0x0F;
      if (c == 0xE0) lo = 0xA0;
      if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      n = 4; v = c & 0x07;
      if (c == 0xF0) lo = 0x90;
      if (c == 0xF4) hi = 0x8F;
    } else { *r = 0xFFFD; return 1; }
    if (end - q < n) { *r = 0xFFFD; return 1; }
    for (int i = 1; i < n; i++) {
      unsigned b = q[i];
      if (b < (i == 1 ? lo : 0x80) || b > (i == 1 ? hi : 0xBF)) { *r = 0xFFFD; return 1; }
      v = (v << 6) | (b & 0x3F);
    }
    *r = v;
    return n;
  }
  static int hex4(const unsigned char* q) {
    int v = 0;
    for (int i = 0; i < 4; i++) {
      int c = q[i], d;
      if (c >= '0' && c <= '9') d = c - '0';
      else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
      else return -1;
      v = v * 16 + d;
    }
    return v;
  }
  // a JSON string at p (p at '"'); out may be null (validate only)
  bool str(std::string* out) {
    if (p >= e || *p != '"') return syntax();
    p++;
    if (out) out->clear();
    {  // fast path: plain printable ASCII up to the closing quote
      const unsigned char* q = p;
      while (q < e && *q != '"' && *q != '\\' && *q >= 0x20 && *q < 0x80) q++;
      if (q < e && *q == '"') {
        if (out) out->assign(reinterpret_cast<const char*>(p), size_t(q - p));
        p = q + 1;
        return true;
      }
      if (out) out->assign(reinterpret_cast<const char*>(p), size_t(q - p));
      p = q;
    }
    while (true) {
      if (p >= e) return syntax();
      unsigned c = *p;
      if (c == '"') { p++; return true; }
      if (c < 0x20) return syntax();
      if (c == '\\') {
        if (e - p < 2) return syntax();
        unsigned k = p[1];
        p += 2;
        char simple = 0;
        switch (k) {
          case '"': simple = '"'; break;
          case '\\': simple = '\\'; break;
          case '/': simple = '/'; break;
          case 'b': simple = '\b'; break;
          case 'f': simple = '\f'; break;
          case 'n': simple = '\n'; break;
          case 'r': simple = '\r'; break;
          case 't': simple = '\t'; break;
          case 'u': {
            if (e - p < 4) return syntax();
            int u = hex4(p);
            if (u < 0) return syntax();
            p += 4;
            uint32_t r = uint32_t(u);
            if (r >= 0xD800 && r < 0xE000) {  // utf16.IsSurrogate
              uint32_t r2 = 0;
              bool pair = false;
              if (e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                int u2 = hex4(p + 2);
                if (u2 >= 0) {
                  r2 = uint32_t(u2);
                  // utf16.DecodeRune: a valid pair only for high then low
                  if (r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000) {
                    r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
                    p += 6;
                    pair = true;
                  }
                }
              }
              if (!pair) r = 0xFFFD;  // the next escape, if any, is decoded on its own
            }
            if (out) put_utf8(out, r);
            continue;
          }
          default: return syntax();
        }
        if (out) out->push_back(simple);
        continue;
      }
      if (c < 0x80) {
        if (out) out->push_back(char(c));
        p++;
        continue;
      }
      uint32_t r;
      int n = decode_rune(p, e, &r);
      if (out) {
        if (r == 0xFFFD && n == 1) put_utf8(out, 0xFFFD);
        else out->append(reinterpret_cast<const char*>(p), size_t(n));
      }
      p += n;
    }
  }
  // JSON number syntax; [b, p) is the literal
  bool number(const unsigned char** b) {
    *b = p;
    if (p < e && *p == '-') p++;
    if (p >= e) return syntax();
    if (*p == '0') p++;
    else if (*p >= '1' && *p <= '9') { while (p < e && *p >= '0' && *p <= '9') p++; }
    else return syntax();
    if (p < e && *p == '.') {
      p++;
      if (p >= e || *p < '0' || *p > '9') return syntax();
      while (p < e && *p >= '0' && *p <= '9') p++;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      p++;
      if (p < e && (*p == '+' || *p == '-')) p++;
      if (p >= e || *p < '0' || *p > '9') return syntax();
      while (p < e && *p >= '0' && *p <= '9') p++;
    }
    return true;
  }
  // validate and skip any value
  bool skip(int depth = 0) {
    if (depth > 10000) return syntax();
    ws();
    if (p >= e) return syntax();
    switch (*p) {
      case '{': {
        p++;
        ws();
        if (p < e && *p == '}') { p++; return true; }
        while (true) {
          ws();
          if (!str(nullptr)) return false;
          ws();
          if (p >= e || *p != ':') return syntax();
          p++;
          if (!skip(depth + 1)) return false;
          ws();
          if (p < e && *p == ',') { p++; continue; }
          if (p < e && *p == '}') { p++; return true; }
          return syntax();
        }
      }
      case '[': {
        p++;
        ws();
        if (p < e && *p == ']') { p++; return true; }
        while (true) {
          if (!skip(depth + 1)) return false;
          ws();
          if (p < e && *p == ',') { p++; continue; }
          if (p < e && *p == ']') { p++; return true; }
          return syntax();
        }
      }
      case '"': return str(nullptr);
      case 't': return lit("true");
      case 'f': return lit("false");
      case 'n': return lit("null");
      default: {
        const unsigned char* b;
        return number(&b);
      }
    }
  }
  bool peek_null() {
    ws();
    return p < e && *p == 'n';
  }
  // field decoders: each consumes exactly one value
  bool dec_string(std::string* out) {
    ws();
    if (p >= e) return syntax();
    if (*p == '"') return str(out);
    if (*p == 'n') return lit("null");  // null: unchanged
    type_err();
    return skip();
  }
  bool dec_int(int64_t* out) {
    ws();
    if (p >= e) return syntax();
    if (*p == 'n') return lit("null");
    if (*p == '-' || (*p >= '0' && *p <= '9')) {
      const unsigned char* b;
      if (!number(&b)) return false;
      // strconv.ParseInt(s, 10, 64): digits only, in range
      const unsigned char* q = b;
      bool neg = false;
      if (*q == '-') { neg = true; q++; }
      unsigned long long v = 0;
      bool ok = q < p;
      for (; q < p && ok; q++) {
        if (*q < '0' || *q > '9') { ok = false; break; }
        unsigned d = *q - '0';
        if (v > (~0ull - d) / 10) { ok = false; break; }
        v = v * 10 + d;
      }
      if (ok && (neg ? v > (1ull << 63) : v > (1ull << 63) - 1)) ok = false;
      if (!ok) { type_err(); return true; }
      *out = neg ? int64_t(0 - v) : int64_t(v);
      return true;
    }
    type_err();
    return skip();
  }
  bool dec_bool(bool* out) {
    ws();
    if (p >= e) return syntax();
    if (*p == 't') { if (!lit("true")) return false; *out = true; return true; }
    if (*p == 'f') { if (!lit("false")) return false; *out = false; return true; }
    if (*p == 'n') return lit("null");
    type_err();
    return skip();
  }
  // generic Go-slice array decode; elem(T* slot) decodes one element into slot
  template <class T, class F, class Z>
  bool dec_slice(GoSlice<T>* s, F elem, Z zero) {
    ws();
    if (p >= e) return syntax();
    if (*p == 'n') {
      if (!lit("null")) return false;
      s->set_nil();
      return true;
    }
    if (*p != '[') {
      type_err();
      return skip();
    }
    p++;
    size_t i = 0;
    ws();
    if (p < e && *p == ']') {
      p++;
    } else {
      while (true) {
        if (i >= s->backing.size()) {  // grow: cap + cap/2, >= 4; copies len elements
          size_t cap = s->backing.size(), nc = cap + cap / 2;
          if (nc < 4) nc = 4;
          std::vector<T> nb(nc, zero());
          for (size_t k = 0; k < s->len; k++) nb[k] = s->backing[k];
          s->backing.swap(nb);
        }
        if (i >= s->len) s->len = i + 1;
        if (!elem(&s->backing[i])) return false;
        i++;
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == ']') { p++; break; }
        return syntax();
      }
    }
    s->nil = false;
    if (i < s->len) s->len = i;
    if (i == 0) {  // reflect.MakeSlice(t, 0, 0)
      s->backing.clear();
      s->len = 0;
    }
    return true;
  }
  bool dec_strings(GoSlice<std::string>* s) {
    return dec_slice(s, [this](std::string* x) { return dec_string(x); },
                     [] { return std::string(); });
  }
};

// encoding/json key matching against one field tag (fold.go of Go 1.8)
bool key_matches(const std::string& key, const char* name) {
  const size_t n = std::strlen(name);
  if (key.size() == n && std::memcmp(key.data(), name, n) == 0) return true;
  bool special = false;
  for (size_t i = 0; i < n; i++) {
    char u = char(name[i] & ~0x20);
    if (u == 'K' || u == 'S') special = true;
  }
  const unsigned char* t = reinterpret_cast<const unsigned char*>(key.data());
  const unsigned char* te = t + key.size();
  for (size_t i = 0; i < n; i++) {
    const unsigned char sb = static_cast<unsigned char>(name[i]);
    if (t >= te) return false;
    if (*t < 0x80) {
      if (sb != *t) {
        const unsigned char su = sb & 0xDF;
        if (!(su >= 'A' && su <= 'Z') || su != (*t & 0xDF)) return false;
      }
      t++;
      continue;
    }
    if (!special) return false;
    // K (E2 84 AA) for k/K, ſ (C5 BF) for s/S
    if ((sb == 'k' || sb == 'K') && te - t >= 3 && t[0] == 0xE2 && t[1] == 0x84 && t[2] == 0xAA) {
      t += 3;
      continue;
    }
    if ((sb == 's' || sb == 'S') && te - t >= 2 && t[0] == 0xC5 && t[1] == 0xBF) {
      t += 2;
      continue;
    }
    return false;
  }
  return t == te;
}

// the field a key selects: an exact match first, else the first fold match
int pick_field(const std::string& key, const char* const* names, int n) {
  for (int i = 0; i < n; i++)
    if (key == names[i]) return i;
  for (int i = 0; i < n; i++)
    if (key_matches(key, names[i])) return i;
  return -1;
}

// decode an object, calling field(i) for known keys (i = index into names)
template <class F>
bool dec_object(Dec& d, const char* const* names, int n, F field) {
  d.ws();
  if (d.p >= d.e) return d.syntax();
  if (*d.p != '{') {
    d.type_err();
    return d.skip();
  }
  d.p++;
  d.ws();
  if (d.p < d.e && *d.p == '}') {
    d.p++;
    return true;
  }
  std::string key;
  while (true) {
    d.ws();
    if (!d.str(&key)) return false;
    d.ws();
    if (d.p >= d.e || *d.p != ':') return d.syntax();
    d.p++;
    const int f = pick_field(key, names, n);
    if (f < 0) {
      if (!d.skip()) return false;
    } else if (!field(f)) {
      return false;
    }
    d.ws();
    if (d.p < d.e && *d.p == ',') {
      d.p++;
      continue;
    }
    if (d.p < d.e && *d.p == '}') {
      d.p++;
      return true;
    }
    return d.syntax();
  }
}

const char* const kRuleFields[] = {"id", "timer", "gids", "nids", "exclude_nids"};
const char* const kJobFields[] = {"id",        "name",  "group",    "cmd",  "user",
                                  "rules",     "pause", "timeout",  "parallels",
                                  "retry",     "interval", "kind",  "avg_time",
                                  "fail_notify", "to"};
const char* const kGroupFields[] = {"id", "name", "nids"};

bool dec_rule(Dec& d, PRule* r) {
  return dec_object(d, kRuleFields, 5, [&](int f) {
    switch (f) {
      case 0: return d.dec_string(&r->id);
      case 1: return d.dec_string(&r->timer);
      case 2: return d.dec_strings(&r->gids);
      case 3: return d.dec_strings(&r->nids);
      default: return d.dec_strings(&r->ex);
    }
  });
}

bool dec_job(Dec& d, PJob* j) {
  return dec_object(d, kJobFields, 15, [&](int f) {
    switch (f) {
      case 0: return d.dec_string(&j->id);
      case 1: return d.dec_string(&j->name);
      case 2: return d.dec_string(&j->group);
      case 3: return d.dec_string(&j->cmd);
      case 4: return d.dec_string(&j->user);
      case 5:
        return d.dec_slice(
            &j->rules,
            [&](int32_t* slot) {
              if (d.peek_null()) {  // *JobRule <- null: nil
                if (!d.lit("null")) return false;
                *slot = -1;
                return true;
              }
              d.ws();
              if (d.p < d.e && *d.p != '{') {  // not an object: type error, skip it
                d.type_err();
                return d.skip();
              }
              if (*slot < 0) {  // indirect(): allocate a new JobRule
                j->pool.emplace_back();
                *slot = int32_t(j->pool.size()) - 1;
              }
              return dec_rule(d, &j->pool[size_t(*slot)]);
            },
            [] { return int32_t(-1); });
      case 6: return d.dec_bool(&j->pause);
      case 7: return d.dec_int(&j->timeout);
      case 8: return d.dec_int(&j->parallels);
      case 9: return d.dec_int(&j->retry);
      case 10: return d.dec_int(&j->interval);
      case 11: return d.dec_int(&j->kind);
      case 12: return d.dec_int(&j->avg_time);
      case 13: return d.dec_bool(&j->fail_notify);
      default: return d.dec_strings(&j->to);
    }
  });
}

bool dec_group(Dec& d, PGroup* g) {
  return dec_object(d, kGroupFields, 3, [&](int f) {
    switch (f) {
      case 0: return d.dec_string(&g->id);
      case 1: return d.dec_string(&g->name);
      default: return d.dec_strings(&g->nids);
    }
  });
}

// json.Unmarshal(doc, v): kOk, kSyntax or kType
template <class T, class F>
int unmarshal(const char* doc, size_t len, T* v, F dec) {
  Dec d;
  d.p = reinterpret_cast<const unsigned char*>(doc);
  d.e = d.p + len;
  // Go validates the whole value first (checkValid) and then decodes; since
  // GetJobs/GetGroups discard a value on either kind of error, one pass that
  // validates everything it consumes (unknown and mistyped values included)
  // decides the same
  d.ws();
  if (d.p < d.e && *d.p == 'n') {  // null: v unchanged
    if (!d.lit("null")) return kSyntax;
  } else if (!dec(d, v)) {
    return kSyntax;
  }
  d.ws();
  if (d.p != d.e) return kSyntax;
  return d.err;
}

std::vector<std::string> visible(const GoSlice<std::string>& s) {
  return std::vector<std::string>(s.backing.begin(), s.backing.begin() + long(s.len));
}

template <class W>
void parallel_for(size_t n, int nthreads, W work) {
  if (nthreads < 1) nthreads = 1;
  if (size_t(nthreads) > n / 256 + 1) nthreads = int(n / 256 + 1);
  std::vector<std::thread> th;
  const size_t chunk = (n + size_t(nthreads) - 1) / size_t(nthreads);
  for (int t = 0; t < nthreads; t++) {
    size_t lo = size_t(t) * chunk, hi = std::min(n, lo + chunk);
    if (lo >= hi) break;
    th.emplace_back([=] { for (size_t i = lo; i < hi; i++) work(i); });
  }
  for (auto& x : th) x.join();
}

std::vector<const char*> cstrs(const std::vector<std::string>& v) {
  std::vector<const char*> o;
  for (auto& s : v) o.push_back(s.c_str());
  return o;
}

}  // namespace

extern "C" {

int cg_jobset_ingest_groups(cg_jobset* js, const char* const* docs, const size_t* lens, size_t n,
                            int nthreads, int32_t* status) {
  if (!js || (n && (!docs || !lens))) return cg_fail(CG_EINVAL, "cg_jobset_ingest_groups: null");
  std::vector<PGroup> g(n);
  std::vector<int32_t> st(n, CG_INGEST_OK);
  parallel_for(n, nthreads, [&](size_t i) {
    if (unmarshal(docs[i] ? docs[i] : "", docs[i] ? lens[i] : 0, &g[i], dec_group) != kOk) {
      st[i] = CG_INGEST_UNMARSHAL;
      return;
    }
    bool nul = g[i].id.find('\0') != std::string::npos;
    for (size_t q = 0; q < g[i].nids.len && !nul; q++)
      nul = g[i].nids.backing[q].find('\0') != std::string::npos;
    if (nul) st[i] = CG_INGEST_UNSUPPORTED;
  });
  // groups[group.ID] = group: the last value of an ID wins (group.go:53-60)
  std::unordered_map<std::string, size_t> last;
  for (size_t i = 0; i < n; i++)
    if (st[i] == CG_INGEST_OK) last[g[i].id] = i;
  for (size_t i = 0; i < n; i++) {
    if (st[i] != CG_INGEST_OK) continue;
    if (last[g[i].id] != i) {
      st[i] = CG_INGEST_REPLACED;
      continue;
    }
    auto nids = visible(g[i].nids);
    auto c = cstrs(nids);
    int rc = cg_jobset_add_group(js, g[i].id.c_str(), c.data(), c.size());
    if (rc) return rc;
  }
  if (status) std::copy(st.begin(), st.end(), status);
  return CG_OK;
}

int cg_jobset_ingest_jobs(cg_jobset* js, const char* const* docs, const size_t* lens, size_t n,
                          int nthreads, int32_t* status) {
  if (!js || (n && (!docs || !lens))) return cg_fail(CG_EINVAL, "cg_jobset_ingest_jobs: null");
  std::vector<PJob> jobs(n);
  std::vector<int32_t> st(n, CG_INGEST_OK);
  std::vector<std::vector<cg_schedule>> sched(n);
  parallel_for(n, nthreads, [&](size_t i) {
    PJob& j = jobs[i];
    if (unmarshal(docs[i] ? docs[i] : "", docs[i] ? lens[i] : 0, &j, dec_job) != kOk) {
      st[i] = CG_INGEST_UNMARSHAL;
      return;
    }
    // Job.Valid -> ValidRules: the first failing rule decides (job.go:683-690)
    for (size_t k = 0; k < j.rules.len; k++) {
      const int32_t r = j.rules.backing[k];
      if (r < 0) {  // nil *JobRule: r.Valid() dereferences it
        st[i] = CG_INGEST_PANIC;
        return;
      }
      const PRule& rule = j.pool[size_t(r)];
      if (rule.timer.empty()) {  // ErrNilRule
        st[i] = CG_INGEST_INVALID;
        return;
      }
      cg_schedule s{};
      if (cg_parse(CG_PARSE_DEFAULT, rule.timer.data(), rule.timer.size(), &s, nullptr, 0) != CG_OK) {
        st[i] = CG_INGEST_INVALID;
        return;
      }
      sched[i].push_back(s);
    }
    if (j.kind == CG_JOB_ALONE) j.parallels = 1;  // alone(), job.go:378-382
    // IDs cross the C-ABI as NUL-terminated strings
    auto has_nul = [](const std::string& x) { return x.find('\0') != std::string::npos; };
    bool nul = has_nul(j.id);
    for (size_t k = 0; k < j.rules.len && !nul; k++) {
      const PRule& r = j.pool[size_t(j.rules.backing[k])];
      nul = has_nul(r.id);
      for (const auto* sl : {&r.gids, &r.nids, &r.ex})
        for (size_t q = 0; q < sl->len && !nul; q++) nul = has_nul(sl->backing[q]);
    }
    if (nul) st[i] = CG_INGEST_UNSUPPORTED;
  });
  // jobs[job.ID] = job: the last valid value of an ID wins (job.go:353-364)
  std::unordered_map<std::string_view, size_t> last;
  last.reserve(n);
  for (size_t i = 0; i < n; i++)
    if (st[i] == CG_INGEST_OK) last[jobs[i].id] = i;
  js->node_idx.reserve(js->node_idx.size() + n / 4);
  for (size_t i = 0; i < n; i++) {
    if (st[i] != CG_INGEST_OK) continue;
    if (last.find(jobs[i].id)->second != i) {
      st[i] = CG_INGEST_REPLACED;
      continue;
    }
    PJob& j = jobs[i];
    // cg_jobset_add_job + cg_jobset_add_rule, interning straight from the
    // decoded strings
    js->job_ids.push_back(j.id);  // (j.id backs a key of `last`: copied, not moved)
    js->job_pause.push_back(j.pause ? 1 : 0);
    js->job_first_rule.push_back(int32_t(js->rule_ids.size()));
    js->job_kind.push_back(int32_t(j.kind));
    js->job_avg.push_back(j.avg_time);
    js->job_parallels.push_back(j.parallels);
    const int32_t job = int32_t(js->job_ids.size()) - 1;
    for (size_t k = 0; k < j.rules.len; k++) {
      PRule& r = j.pool[size_t(j.rules.backing[k])];
      js->rule_ids.push_back(std::move(r.id));
      js->rule_job.push_back(job);
      std::vector<int32_t> a(r.gids.len), b(r.nids.len), c(r.ex.len);
      for (size_t q = 0; q < r.gids.len; q++) a[q] = js->group(r.gids.backing[q]);
      for (size_t q = 0; q < r.nids.len; q++) b[q] = js->node(r.nids.backing[q]);
      for (size_t q = 0; q < r.ex.len; q++) c[q] = js->node(r.ex.backing[q]);
      js->r_gids.push_back(std::move(a));
      js->r_nids.push_back(std::move(b));
      js->r_ex.push_back(std::move(c));
      js->rule_sched.push_back(sched[i][k]);
      js->rule_has_sched.push_back(1);
    }
  }
  if (status) std::copy(st.begin(), st.end(), status);
  return CG_OK;
}

int cg_jobset_schedules(const cg_jobset* js, cg_schedule* out, size_t cap) {
  if (!js || (cap && !out)) return cg_fail(CG_EINVAL, "cg_jobset_schedules: null");
  const size_t R = js->rule_ids.size();
  for (size_t r = 0; r < R; r++)
    if (!js->rule_has_sched[r])
      return cg_fail(CG_EINVAL, "rule " + std::to_string(r) +
                                    " was added without a timer (cg_jobset_add_rule)");
  for (size_t r = 0; r < R && r < cap; r++) out[r] = js->rule_sched[r];
  return int(R > size_t(INT32_MAX) ? INT32_MAX : R);
}

int cg_jobset_job_meta(const cg_jobset* js, int32_t* kind, int64_t* avg_time_ms,
                       int64_t* parallels, size_t cap) {
  if (!js) return cg_fail(CG_EINVAL, "cg_jobset_job_meta: null");
  const size_t J = js->job_ids.size();
  for (size_t j = 0; j < J && j < cap; j++) {
    if (kind) kind[j] = js->job_kind[j];
    if (avg_time_ms) avg_time_ms[j] = js->job_avg[j];
    if (parallels) parallels[j] = js->job_parallels[j];
  }
  return int(J > size_t(INT32_MAX) ? INT32_MAX : J);
}

const char* cg_jobset_job_id(const cg_jobset* js, int32_t job) {
  if (!js || job < 0 || job >= int32_t(js->job_ids.size())) return nullptr;
  return js->job_ids[size_t(job)].c_str();
}

const char* cg_jobset_group_id(const cg_jobset* js, int32_t group) {
  if (!js || group < 0 || group >= int32_t(js->group_ids.size())) return nullptr;
  return js->group_ids[size_t(group)].c_str();
}

const char* cg_jobset_rule_id(const cg_jobset* js, int32_t rule) {
  if (!js || rule < 0 || rule >= int32_t(js->rule_ids.size())) return nullptr;
  return js->rule_ids[size_t(rule)].c_str();
}

}  // extern "C"
