// Host ingest (include/hstream_ingest.h): JSON record values of a poll batch
// into the columnar hsg_batch, with the GROUP BY key dictionary-encoded under
// Aeson Value equality.
//
// Reference behaviour restated (per record, in the reference's order):
//   value decode              Processor.hs:192-204 (Aeson Object; failure aborts
//                             the record, runTask's catch at Processor.hs:140-143)
//   GROUP BY key              Codegen.hs:485-487, getFieldByName throws when the
//                             field is absent (Internal/Codegen.hs:41-49)
//   aggregated field reads    Codegen.hs:412-461 (absent: accumulator unchanged;
//                             COUNT(col) counts any present value, null too;
//                             SUM/MIN/MAX need a Number, anything else throws)
// Key identity is Aeson's Value equality: numbers compare as Data.Scientific
// (the exact decimal value: 1 == 1.0 == 1E0 == 10e-1), strings by their
// unescaped text, objects as maps (member order irrelevant), arrays by
// element. The dictionary keys on a canonical byte form of that equality
// class and keeps, per key, the Aeson encoding of its first spelling.
//
// Decoding fans out over host threads (contiguous record ranges); ids are
// then handed out in record order, so the ids are those a sequential pass
// would give.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/hstream_gpu.h"
#include "../../include/hstream_ingest.h"

namespace {

// ---------------------------------------------------------------------------
// JSON scanning
// ---------------------------------------------------------------------------
struct Cur {
  const char *p, *e;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool eat(char c) {
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
};

void put_utf8(std::string &o, uint32_t cp) {
  if (cp < 0x80) {
    o.push_back((char)cp);
  } else if (cp < 0x800) {
    o.push_back((char)(0xC0 | (cp >> 6)));
    o.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    o.push_back((char)(0xE0 | (cp >> 12)));
    o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    o.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    o.push_back((char)(0xF0 | (cp >> 18)));
    o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    o.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

int hexv(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool hex4(Cur &c, uint32_t &v) {
  if (c.e - c.p < 4) return false;
  v = 0;
  for (int i = 0; i < 4; ++i) {
    int h = hexv(c.p[i]);
    if (h < 0) return false;
    v = v * 16 + (uint32_t)h;
  }
  c.p += 4;
  return true;
}

// A string at c.p ('"'): raw span [s, s + n) between the quotes and whether it
// holds escapes. No unescaping.
bool string_span(Cur &c, const char *&s, size_t &n, bool &esc) {
  if (!c.eat('"')) return false;
  s = c.p;
  esc = false;
  while (c.p < c.e) {
    const char ch = *c.p;
    if (ch == '"') {
      n = (size_t)(c.p - s);
      ++c.p;
      return true;
    }
    if (ch == '\\') {
      esc = true;
      if (c.e - c.p < 2) return false;
      c.p += 2;
      continue;
    }
    if ((unsigned char)ch < 0x20) return false;  // raw control characters are not JSON
    ++c.p;
  }
  return false;
}

// Unescape a raw string body into o.
bool unescape(const char *s, size_t n, std::string &o) {
  Cur c{s, s + n};
  while (c.p < c.e) {
    const char ch = *c.p++;
    if (ch != '\\') {
      o.push_back(ch);
      continue;
    }
    if (c.p >= c.e) return false;
    const char x = *c.p++;
    switch (x) {
      case '"': o.push_back('"'); break;
      case '\\': o.push_back('\\'); break;
      case '/': o.push_back('/'); break;
      case 'b': o.push_back('\b'); break;
      case 'f': o.push_back('\f'); break;
      case 'n': o.push_back('\n'); break;
      case 'r': o.push_back('\r'); break;
      case 't': o.push_back('\t'); break;
      case 'u': {
        uint32_t v;
        if (!hex4(c, v)) return false;
        if (v >= 0xD800 && v < 0xDC00) {  // high surrogate: a low one must follow
          uint32_t lo;
          if (c.e - c.p < 6 || c.p[0] != '\\' || c.p[1] != 'u') return false;
          c.p += 2;
          if (!hex4(c, lo) || lo < 0xDC00 || lo >= 0xE000) return false;
          v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
        } else if (v >= 0xDC00 && v < 0xE000) {
          return false;
        }
        put_utf8(o, v);
        break;
      }
      default: return false;
    }
  }
  return true;
}

// A JSON number literal, split for exact (Scientific) handling.
struct Num {
  const char *s, *t;    // the literal
  bool neg;
  const char *ip, *ie;  // integer digits
  const char *fp, *fe;  // fraction digits
  int64_t exp;          // exponent part (saturated)
};

bool parse_number(Cur &c, Num &n) {
  n.s = c.p;
  n.neg = c.eat('-');
  n.ip = c.p;
  if (c.p < c.e && *c.p == '0') {
    ++c.p;
  } else {
    if (c.p >= c.e || *c.p < '1' || *c.p > '9') return false;
    while (c.p < c.e && *c.p >= '0' && *c.p <= '9') ++c.p;
  }
  n.ie = c.p;
  n.fp = n.fe = c.p;
  if (c.eat('.')) {
    n.fp = c.p;
    while (c.p < c.e && *c.p >= '0' && *c.p <= '9') ++c.p;
    n.fe = c.p;
    if (n.fe == n.fp) return false;
  }
  n.exp = 0;
  if (c.p < c.e && (*c.p == 'e' || *c.p == 'E')) {
    ++c.p;
    bool eneg = false;
    if (c.p < c.e && (*c.p == '+' || *c.p == '-')) eneg = *c.p++ == '-';
    const char *d0 = c.p;
    int64_t v = 0;
    while (c.p < c.e && *c.p >= '0' && *c.p <= '9') {
      if (v < (int64_t)1e15) v = v * 10 + (*c.p - '0');
      ++c.p;
    }
    if (c.p == d0) return false;
    n.exp = eneg ? -v : v;
  }
  n.t = c.p;
  return true;
}

// Normalised decimal: value = (neg ? -1 : 1) * D * 10^e, D without leading or
// trailing zeros ("" = zero).
struct Dec {
  std::string d;
  int64_t e = 0;
  bool neg = false;
  int64_t spelled_exp = 0;  // exponent of the literal's own coefficient (Aeson keeps it)
};

void normalise(const Num &n, Dec &x) {
  x.d.clear();
  bool lead = true;  // leading zeros are dropped as they come
  for (const char *q = n.ip; q < n.ie; ++q)
    if (!(lead && *q == '0')) lead = false, x.d.push_back(*q);
  for (const char *q = n.fp; q < n.fe; ++q)
    if (!(lead && *q == '0')) lead = false, x.d.push_back(*q);
  x.spelled_exp = n.exp - (int64_t)(n.fe - n.fp);
  int64_t e = x.spelled_exp;
  while (!x.d.empty() && x.d.back() == '0') {
    x.d.pop_back();
    ++e;
  }
  x.e = x.d.empty() ? 0 : e;
  x.neg = n.neg && !x.d.empty();  // -0 == 0
}

bool skip_value(Cur &c, int depth = 0);

bool skip_value(Cur &c, int depth) {
  if (depth > 512) return false;
  c.ws();
  if (c.p >= c.e) return false;
  const char ch = *c.p;
  if (ch == '"') {
    const char *s;
    size_t n;
    bool esc;
    return string_span(c, s, n, esc);
  }
  if (ch == '{' || ch == '[') {
    const char close = ch == '{' ? '}' : ']';
    ++c.p;
    c.ws();
    if (c.eat(close)) return true;
    for (;;) {
      if (ch == '{') {
        c.ws();
        const char *s;
        size_t n;
        bool esc;
        if (!string_span(c, s, n, esc)) return false;
        c.ws();
        if (!c.eat(':')) return false;
      }
      if (!skip_value(c, depth + 1)) return false;
      c.ws();
      if (c.eat(close)) return true;
      if (!c.eat(',')) return false;
    }
  }
  if (ch == 't') {
    if (c.e - c.p >= 4 && !memcmp(c.p, "true", 4)) return c.p += 4, true;
    return false;
  }
  if (ch == 'f') {
    if (c.e - c.p >= 5 && !memcmp(c.p, "false", 5)) return c.p += 5, true;
    return false;
  }
  if (ch == 'n') {
    if (c.e - c.p >= 4 && !memcmp(c.p, "null", 4)) return c.p += 4, true;
    return false;
  }
  Num n;
  return parse_number(c, n);
}

// ---------------------------------------------------------------------------
// canonical bytes of a value's equality class
//   z null | t true | f false | n0 zero | n<+|-><digits>e<exp>;
//   s<u32 len><utf8> | [ values ] | { (s-key value)* sorted by key, last duplicate wins }
// ---------------------------------------------------------------------------
void put_u32(std::string &o, uint32_t v) { o.append((const char *)&v, 4); }

// form: when given, one char per number of the value in canonical order --
// 'i' if aeson prints it as an integer (its literal's exponent in [0, 1024]),
// 'd' if in Scientific's Generic form (aeson_number below). Equal values print
// alike iff their forms are equal: the form picks the spelling of a key.
bool canon_value(Cur &c, std::string &o, Dec &tmp, int depth = 0, std::string *form = nullptr);

bool canon_string(Cur &c, std::string &o) {
  const char *s;
  size_t n;
  bool esc;
  if (!string_span(c, s, n, esc)) return false;
  o.push_back('s');
  const size_t at = o.size();
  put_u32(o, 0);
  if (esc) {
    if (!unescape(s, n, o)) return false;
  } else {
    o.append(s, n);
  }
  const uint32_t len = (uint32_t)(o.size() - at - 4);
  memcpy(&o[at], &len, 4);
  return true;
}

void canon_number(const Dec &x, std::string &o) {
  if (x.d.empty()) {
    o.append("n0");
    return;
  }
  o.push_back('n');
  o.push_back(x.neg ? '-' : '+');
  o.append(x.d);
  o.push_back('e');
  char b[24];
  int k = 0;
  uint64_t m = x.e < 0 ? (uint64_t)0 - (uint64_t)x.e : (uint64_t)x.e;
  do {
    b[k++] = (char)('0' + m % 10);
    m /= 10;
  } while (m);
  if (x.e < 0) o.push_back('-');
  while (k) o.push_back(b[--k]);
  o.push_back(';');
}

bool canon_value(Cur &c, std::string &o, Dec &tmp, int depth, std::string *form) {
  if (depth > 512) return false;
  c.ws();
  if (c.p >= c.e) return false;
  const char ch = *c.p;
  if (ch == '"') return canon_string(c, o);
  if (ch == '[') {
    ++c.p;
    o.push_back('[');
    c.ws();
    if (!c.eat(']')) {
      for (;;) {
        if (!canon_value(c, o, tmp, depth + 1, form)) return false;
        c.ws();
        if (c.eat(']')) break;
        if (!c.eat(',')) return false;
      }
    }
    o.push_back(']');
    return true;
  }
  if (ch == '{') {
    ++c.p;
    struct Mem {
      std::string key, val, form;
    };
    std::vector<Mem> mem;
    c.ws();
    if (!c.eat('}')) {
      for (;;) {
        c.ws();
        Mem m;
        if (!canon_string(c, m.key)) return false;
        c.ws();
        if (!c.eat(':')) return false;
        if (!canon_value(c, m.val, tmp, depth + 1, form ? &m.form : nullptr)) return false;
        mem.push_back(std::move(m));
        c.ws();
        if (c.eat('}')) break;
        if (!c.eat(',')) return false;
      }
    }
    // a map: sorted by key; a repeated key keeps its last value
    std::stable_sort(mem.begin(), mem.end(), [](const Mem &a, const Mem &b) { return a.key < b.key; });
    o.push_back('{');
    for (size_t i = 0; i < mem.size(); ++i) {
      if (i + 1 < mem.size() && mem[i + 1].key == mem[i].key) continue;
      o.append(mem[i].key);
      o.append(mem[i].val);
      if (form) form->append(mem[i].form);
    }
    o.push_back('}');
    return true;
  }
  if (ch == 't' || ch == 'f' || ch == 'n') {
    const char *s0 = c.p;
    if (!skip_value(c, depth + 1)) return false;
    o.push_back(*s0 == 'n' ? 'z' : *s0);
    return true;
  }
  Num n;
  if (!parse_number(c, n)) return false;
  normalise(n, tmp);
  canon_number(tmp, o);
  if (form) form->push_back(tmp.spelled_exp >= 0 && tmp.spelled_exp <= 1024 ? 'i' : 'd');
  return true;
}

// ---------------------------------------------------------------------------
// Aeson's encoding of a value (aeson 1.4, lts-16.21): numbers whose literal
// exponent is in [0, 1024] print as integers, others through Scientific's
// formatScientific Generic (fixed for 0.1 <= |x| < 10^7, else d.ddde<n>);
// strings escape '"', '\\', \n \r \t and other controls as \u00XX.
// ---------------------------------------------------------------------------
void aeson_number(const Dec &x, std::string &o) {
  if (x.d.empty()) {
    // zero: integer form when the literal's exponent is >= 0, else "0.0"
    o.append(x.spelled_exp >= 0 && x.spelled_exp <= 1024 ? "0" : "0.0");
    return;
  }
  if (x.neg) o.push_back('-');
  if (x.spelled_exp >= 0 && x.spelled_exp <= 1024) {
    o.append(x.d);
    for (int64_t i = 0; i < x.e; ++i) o.push_back('0');
    return;
  }
  const int64_t E = (int64_t)x.d.size() + x.e;  // value = 0.D * 10^E
  if (E < 0 || E > 7) {
    o.push_back(x.d[0]);
    o.push_back('.');
    if (x.d.size() > 1) o.append(x.d, 1, std::string::npos);
    else o.push_back('0');
    o.push_back('e');
    o.append(std::to_string(E - 1));
    return;
  }
  if (E == 0) {
    o.append("0.");
    o.append(x.d);
    return;
  }
  // E in [1, 7]: E digits before the point (zero-padded), the rest after
  for (int64_t i = 0; i < E; ++i) o.push_back(i < (int64_t)x.d.size() ? x.d[(size_t)i] : '0');
  o.push_back('.');
  if ((int64_t)x.d.size() > E) o.append(x.d, (size_t)E, std::string::npos);
  else o.push_back('0');
}

void aeson_string(const std::string &s, std::string &o) {
  static const char hx[] = "0123456789abcdef";
  o.push_back('"');
  for (unsigned char ch : s) {
    if (ch == '\\') o.append("\\\\");
    else if (ch == '"') o.append("\\\"");
    else if (ch >= 0x20) o.push_back((char)ch);
    else if (ch == '\n') o.append("\\n");
    else if (ch == '\r') o.append("\\r");
    else if (ch == '\t') o.append("\\t");
    else {
      o.append("\\u00");
      o.push_back(hx[ch >> 4]);
      o.push_back(hx[ch & 15]);
    }
  }
  o.push_back('"');
}

bool aeson_value(Cur &c, std::string &o, int depth = 0) {
  if (depth > 512) return false;
  c.ws();
  if (c.p >= c.e) return false;
  const char ch = *c.p;
  if (ch == '"') {
    const char *s;
    size_t n;
    bool esc;
    if (!string_span(c, s, n, esc)) return false;
    std::string u;
    if (esc) {
      if (!unescape(s, n, u)) return false;
    } else {
      u.assign(s, n);
    }
    aeson_string(u, o);
    return true;
  }
  if (ch == '[') {
    ++c.p;
    o.push_back('[');
    c.ws();
    bool first = true;
    if (!c.eat(']')) {
      for (;;) {
        if (!first) o.push_back(',');
        first = false;
        if (!aeson_value(c, o, depth + 1)) return false;
        c.ws();
        if (c.eat(']')) break;
        if (!c.eat(',')) return false;
      }
    }
    o.push_back(']');
    return true;
  }
  if (ch == '{') {
    ++c.p;
    std::vector<std::pair<std::string, std::string>> mem;  // unescaped key, encoded value
    c.ws();
    if (!c.eat('}')) {
      for (;;) {
        c.ws();
        const char *s;
        size_t n;
        bool esc;
        if (!string_span(c, s, n, esc)) return false;
        std::pair<std::string, std::string> m;
        if (esc) {
          if (!unescape(s, n, m.first)) return false;
        } else {
          m.first.assign(s, n);
        }
        c.ws();
        if (!c.eat(':')) return false;
        if (!aeson_value(c, m.second, depth + 1)) return false;
        mem.push_back(std::move(m));
        c.ws();
        if (c.eat('}')) break;
        if (!c.eat(',')) return false;
      }
    }
    std::stable_sort(mem.begin(), mem.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    o.push_back('{');
    bool first = true;
    for (size_t i = 0; i < mem.size(); ++i) {
      if (i + 1 < mem.size() && mem[i + 1].first == mem[i].first) continue;
      if (!first) o.push_back(',');
      first = false;
      aeson_string(mem[i].first, o);
      o.push_back(':');
      o.append(mem[i].second);
    }
    o.push_back('}');
    return true;
  }
  if (ch == 't' || ch == 'f' || ch == 'n') {
    const char *s0 = c.p;
    if (!skip_value(c, depth + 1)) return false;
    o.append(s0, (size_t)(c.p - s0));
    return true;
  }
  Num n;
  if (!parse_number(c, n)) return false;
  Dec x;
  normalise(n, x);
  aeson_number(x, o);
  return true;
}

uint64_t hash_bytes(const char *p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xff51afd7ed558ccdull);
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    h = (h ^ w) * 0xbf58476d1ce4e5b9ull;
    h ^= h >> 31;
    p += 8;
    n -= 8;
  }
  uint64_t w = 0;
  memcpy(&w, p, n);
  h = (h ^ w) * 0x94d049bb133111ebull;
  h ^= h >> 29;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 32;
  return h | 1;  // 0 marks an empty slot
}

}  // namespace

// ---------------------------------------------------------------------------
// dictionary
// ---------------------------------------------------------------------------
struct hsg_keydict {
  std::vector<uint64_t> th;   // slot: key hash (0 = empty)
  std::vector<uint32_t> tid;  // slot: id
  std::string canon;          // canonical bytes, id after id
  std::vector<uint64_t> coff{0};
  std::string text;           // Aeson text of the first spelling, id after id
  std::vector<uint64_t> toff{0};
  std::string form;           // canon_value form of the first spelling, id after id
  std::vector<uint64_t> foff{0};
  // alternate spellings: (key id, form) of a key printed unlike its first
  // spelling (1 vs 1.0), their Aeson text by alternate index
  std::unordered_map<std::string, uint32_t> alt_ix;
  std::string alt_text;
  std::vector<uint64_t> alt_off{0};

  // the spelling of a record whose key has id `id` and form `f` (raw JSON of
  // the key for a new alternate's text): id, or HSG_SPELL_ALT | alternate
  int spelling(uint32_t id, const char *f, size_t fn, const char *raw, size_t rn, uint32_t *spell) {
    const uint64_t a = foff[id], b = foff[id + 1];
    if (b - a == fn && (!fn || !memcmp(form.data() + a, f, fn))) {
      *spell = id;
      return HSG_OK;
    }
    std::string k((const char *)&id, 4);
    k.append(f, fn);
    auto it = alt_ix.find(k);
    if (it == alt_ix.end()) {
      if (alt_ix.size() >= (size_t)HSG_SPELL_ALT) return HSG_E_CAPACITY;
      const uint32_t ix = (uint32_t)alt_ix.size();
      Cur cur{raw, raw + rn};
      if (!aeson_value(cur, alt_text)) alt_text.append("null");
      alt_off.push_back(alt_text.size());
      it = alt_ix.emplace(std::move(k), ix).first;
    }
    *spell = HSG_SPELL_ALT | it->second;
    return HSG_OK;
  }

  uint64_t size() const { return coff.size() - 1; }

  void rehash(uint64_t slots) {
    std::vector<uint64_t> nh(slots, 0);
    std::vector<uint32_t> ni(slots, 0);
    const uint64_t m = slots - 1;
    for (uint64_t s = 0; s < th.size(); ++s) {
      if (!th[s]) continue;
      uint64_t q = th[s] & m;
      while (nh[q]) q = (q + 1) & m;
      nh[q] = th[s];
      ni[q] = tid[s];
    }
    th.swap(nh);
    tid.swap(ni);
  }

  // id of canonical bytes c (hash h); -1 = absent. *slot = where it would go
  int64_t find(const char *c, size_t n, uint64_t h, uint64_t *slot) const {
    if (th.empty()) return -1;
    const uint64_t m = th.size() - 1;
    uint64_t q = h & m;
    while (th[q]) {
      if (th[q] == h) {
        const uint32_t id = tid[q];
        const uint64_t a = coff[id], b = coff[id + 1];
        if (b - a == n && !memcmp(canon.data() + a, c, n)) return id;
      }
      q = (q + 1) & m;
    }
    if (slot) *slot = q;
    return -1;
  }

  // insert a new key: canonical bytes + the raw JSON of its first spelling
  // (and that spelling's form)
  int insert(const char *c, size_t n, uint64_t h, const char *raw, size_t rn, uint32_t *id, const char *f = nullptr,
             size_t fn = 0) {
    if (size() >= (uint64_t)HSG_KEY_NONE) return HSG_E_CAPACITY;
    if (2 * (size() + 1) > th.size()) rehash(th.empty() ? 1024 : 2 * th.size());
    uint64_t q = 0;
    find(c, n, h, &q);
    const uint32_t nid = (uint32_t)size();
    th[q] = h;
    tid[q] = nid;
    canon.append(c, n);
    coff.push_back(canon.size());
    Cur cur{raw, raw + rn};
    if (!aeson_value(cur, text)) text.append("null");
    toff.push_back(text.size());
    if (fn) form.append(f, fn);
    else if (!f) {  // (hsg_keydict_encode: the form from the raw text)
      std::string cb, ff;
      Dec tmp;
      Cur c2{raw, raw + rn};
      if (canon_value(c2, cb, tmp, 0, &ff)) form.append(ff);
    }
    foff.push_back(form.size());
    *id = nid;
    return HSG_OK;
  }
};

// ---------------------------------------------------------------------------
// decoder
// ---------------------------------------------------------------------------
struct hsg_decoder {
  std::string key_field;
  bool literal_forms = false;  // valid bit 1: the number's literal has a negative exponent
  struct Col {
    std::string field;
    int32_t type;
    bool numeric;
  };
  std::vector<Col> cols;
};

namespace {

struct Chunk {
  std::string arena;              // canonical key bytes of the chunk's records
  std::vector<uint64_t> koff;     // per record: start in arena (len via next)
  std::string forms;              // per record: the key's form (canon_value), when spellings are asked
  std::vector<uint64_t> fof;      // per record: start in forms (len via next)
  std::vector<uint64_t> khash;
  std::vector<const char *> raw;  // per record: the key's raw JSON span
  std::vector<uint32_t> rawn;
};

bool name_is(const char *s, size_t n, bool esc, const std::string &want, std::string &tmp) {
  if (!esc) return n == want.size() && !memcmp(s, want.data(), n);
  tmp.clear();
  if (!unescape(s, n, tmp)) return false;
  return tmp == want;
}

// One record: fills its columns and the chunk's key entry; returns its status.
int decode_one(const hsg_decoder &dec, const char *s, size_t n, uint64_t i, void *const *cols,
               uint8_t *const *valid, Chunk &ch, Dec &dtmp, std::string &tmp, bool spell) {
  const int C = (int)dec.cols.size();
  for (int c = 0; c < C; ++c) {
    if (valid && valid[c]) valid[c][i] = 0;
    ((int64_t *)cols[c])[i] = 0;
  }
  ch.khash.push_back(0);
  ch.raw.push_back(nullptr);
  ch.rawn.push_back(0);
  ch.koff.push_back(ch.arena.size());
  if (spell) ch.fof.push_back(ch.forms.size());
  const size_t form_at = ch.forms.size();
  Cur cur{s, s + n};
  cur.ws();
  if (!cur.eat('{')) return HSG_DEC_NOT_OBJECT;
  // per column: 0 absent, 1 number (cnum), 2 present non-number
  int state[32];
  Num cnum[32];
  for (int c = 0; c < C; ++c) state[c] = 0;
  bool have_key = false;
  const size_t key_at = ch.arena.size();
  cur.ws();
  if (!cur.eat('}')) {
    for (;;) {
      cur.ws();
      const char *ks;
      size_t kn;
      bool kesc;
      if (!string_span(cur, ks, kn, kesc)) return HSG_DEC_NOT_OBJECT;
      cur.ws();
      if (!cur.eat(':')) return HSG_DEC_NOT_OBJECT;
      cur.ws();
      bool used = false;
      if (name_is(ks, kn, kesc, dec.key_field, tmp)) {
        // the last occurrence wins (Aeson objects are maps)
        ch.arena.resize(key_at);
        if (spell) ch.forms.resize(form_at);
        const char *r0 = cur.p;
        if (!canon_value(cur, ch.arena, dtmp, 0, spell ? &ch.forms : nullptr)) return HSG_DEC_NOT_OBJECT;
        ch.raw.back() = r0;
        ch.rawn.back() = (uint32_t)(cur.p - r0);
        have_key = true;
        used = true;
      }
      int first_col = -1;
      for (int c = 0; c < C; ++c)
        if (name_is(ks, kn, kesc, dec.cols[c].field, tmp)) {
          first_col = c;
          break;
        }
      if (first_col >= 0) {
        Cur probe = cur;
        int st = 2;
        Num num{};
        if (used) {
          // the key field is also aggregated: re-read its span
          probe.p = ch.raw.back();
        }
        probe.ws();
        if (probe.p < probe.e && (*probe.p == '-' || (*probe.p >= '0' && *probe.p <= '9'))) {
          Cur q = probe;
          if (parse_number(q, num)) {
            st = 1;
            if (!used) cur = q;
          }
        }
        if (st == 2 && !used && !skip_value(cur)) return HSG_DEC_NOT_OBJECT;
        for (int c = first_col; c < C; ++c)
          if (c == first_col || name_is(ks, kn, kesc, dec.cols[c].field, tmp)) {
            state[c] = st;
            cnum[c] = num;
          }
        used = true;
      }
      if (!used && !skip_value(cur)) return HSG_DEC_NOT_OBJECT;
      cur.ws();
      if (cur.eat('}')) break;
      if (!cur.eat(',')) return HSG_DEC_NOT_OBJECT;
    }
  }
  cur.ws();
  if (cur.p != cur.e) return HSG_DEC_NOT_OBJECT;
  if (!have_key) return HSG_DEC_NO_KEY;
  int status = HSG_DEC_OK;
  for (int c = 0; c < C && status == HSG_DEC_OK; ++c) {
    if (state[c] == 0) continue;
    const hsg_decoder::Col &col = dec.cols[c];
    if (!col.numeric) {  // COUNT(col): presence only
      valid[c][i] = 1;
      continue;
    }
    if (state[c] != 1) {
      status = HSG_DEC_TYPE;
      break;
    }
    if (col.type == HSG_F64) {
      char buf[512];
      const size_t ln = (size_t)(cnum[c].t - cnum[c].s);
      double v;
      if (ln < sizeof(buf)) {
        memcpy(buf, cnum[c].s, ln);
        buf[ln] = 0;
        v = strtod(buf, nullptr);
      } else {
        std::string big(cnum[c].s, ln);
        v = strtod(big.c_str(), nullptr);
      }
      ((double *)cols[c])[i] = v;
    } else if (cnum[c].fp == cnum[c].fe && cnum[c].exp == 0 && cnum[c].ie - cnum[c].ip <= 18) {
      // plain integer literal of at most 18 digits: always inside int64
      int64_t v = 0;
      for (const char *q = cnum[c].ip; q < cnum[c].ie; ++q) v = v * 10 + (*q - '0');
      ((int64_t *)cols[c])[i] = cnum[c].neg ? -v : v;
    } else {
      normalise(cnum[c], dtmp);
      if (dtmp.d.empty()) {
        ((int64_t *)cols[c])[i] = 0;
      } else {
        if (dtmp.e < 0) {
          status = HSG_DEC_NOT_INTEGRAL;
          break;
        }
        const unsigned __int128 lim = dtmp.neg ? ((unsigned __int128)1 << 63) : (((unsigned __int128)1 << 63) - 1);
        unsigned __int128 v = 0;
        bool over = dtmp.d.size() + (size_t)(dtmp.e > 40 ? 40 : dtmp.e) > 19;
        if (!over) {
          for (char dch : dtmp.d) v = v * 10 + (unsigned)(dch - '0');
          for (int64_t k = 0; k < dtmp.e; ++k) v *= 10;
          over = v > lim;
        }
        if (over) {
          status = HSG_DEC_RANGE;
          break;
        }
        ((int64_t *)cols[c])[i] = dtmp.neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)(uint64_t)v;
      }
    }
    // literal forms: aeson prints this Scientific as an integer iff its
    // exponent (the literal's, e.g. 25e-1 -> -1) is in [0, 1024]
    const int64_t se = cnum[c].exp - (int64_t)(cnum[c].fe - cnum[c].fp);
    valid[c][i] = (uint8_t)(1u | ((dec.literal_forms && (se < 0 || se > 1024)) ? 2u : 0u));
  }
  if (status != HSG_DEC_OK) return status;
  ch.khash.back() = hash_bytes(ch.arena.data() + key_at, ch.arena.size() - key_at);
  return HSG_DEC_OK;
}

}  // namespace

extern "C" int hsg_keydict_create(hsg_keydict **out) {
  if (!out) return HSG_E_INVALID;
  *out = new (std::nothrow) hsg_keydict();
  return *out ? HSG_OK : HSG_E_OOM;
}

extern "C" void hsg_keydict_destroy(hsg_keydict *d) { delete d; }

extern "C" uint64_t hsg_keydict_size(const hsg_keydict *d) { return d ? d->size() : 0; }

extern "C" int hsg_keydict_encode(hsg_keydict *d, const char *json, size_t len, uint32_t *id) {
  if (!d || !json || !id) return HSG_E_INVALID;
  try {
    std::string c;
    Dec tmp;
    Cur cur{json, json + len};
    if (!canon_value(cur, c, tmp)) return HSG_E_INVALID;
    cur.ws();
    if (cur.p != cur.e) return HSG_E_INVALID;
    const uint64_t h = hash_bytes(c.data(), c.size());
    const int64_t f = d->find(c.data(), c.size(), h, nullptr);
    if (f >= 0) {
      *id = (uint32_t)f;
      return HSG_OK;
    }
    return d->insert(c.data(), c.size(), h, json, len, id);
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  }
}

extern "C" int hsg_keydict_text(const hsg_keydict *d, uint32_t id, char *buf, size_t cap, size_t *len) {
  if (!d || !len || id >= d->size()) return HSG_E_INVALID;
  const uint64_t a = d->toff[id], b = d->toff[id + 1];
  *len = (size_t)(b - a);
  if (cap < *len || (!buf && *len)) return HSG_E_CAPACITY;
  if (*len) memcpy(buf, d->text.data() + a, *len);
  return HSG_OK;
}

extern "C" int hsg_decoder_create(const hsg_decoder_config *cfg, hsg_decoder **out) {
  if (!cfg || !out || !cfg->key_field || cfg->n_cols < 0 || cfg->n_cols > 32) return HSG_E_INVALID;
  if (cfg->n_cols && (!cfg->col_fields || !cfg->col_types)) return HSG_E_INVALID;
  try {
    hsg_decoder *d = new hsg_decoder();
    d->key_field = cfg->key_field;
    d->literal_forms = cfg->literal_forms != 0;
    for (int c = 0; c < cfg->n_cols; ++c) {
      if (!cfg->col_fields[c] || (cfg->col_types[c] != HSG_I64 && cfg->col_types[c] != HSG_F64)) {
        delete d;
        return HSG_E_INVALID;
      }
      d->cols.push_back({cfg->col_fields[c], cfg->col_types[c], cfg->col_numeric ? cfg->col_numeric[c] != 0 : true});
    }
    *out = d;
    return HSG_OK;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  }
}

extern "C" void hsg_decoder_destroy(hsg_decoder *d) { delete d; }

extern "C" int hsg_decode_json_spelled(hsg_decoder *dec, hsg_keydict *dict, uint64_t n, const char *buf,
                                       const uint64_t *off, const int64_t *rec_ts, uint32_t *key_id, int64_t *ts,
                                       void *const *cols, uint8_t *const *valid, uint8_t *status, uint64_t *rejected,
                                       uint32_t *spell, int n_threads) {
  if (!dec || !dict || (n && (!buf || !off || !key_id))) return HSG_E_INVALID;
  const int C = (int)dec->cols.size();
  if (C && (!cols || !valid)) return HSG_E_INVALID;
  for (int c = 0; c < C; ++c)
    if (!cols[c] || !valid[c]) return HSG_E_INVALID;
  if (rejected) *rejected = 0;
  if (!n) return HSG_OK;
  try {
    int T = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    if (T < 1) T = 1;
    if (T > 32) T = 32;
    const uint64_t min_per = 2048;
    if ((uint64_t)T > (n + min_per - 1) / min_per) T = (int)((n + min_per - 1) / min_per);
    std::vector<Chunk> chunks((size_t)T);
    std::vector<uint8_t> st_local(status ? 0 : n);
    uint8_t *st = status ? status : st_local.data();
    auto work = [&](int t) {
      const uint64_t lo = n * (uint64_t)t / (uint64_t)T, hi = n * (uint64_t)(t + 1) / (uint64_t)T;
      Chunk &ch = chunks[(size_t)t];
      ch.koff.reserve(hi - lo + 1);
      if (spell) ch.fof.reserve(hi - lo + 1);
      ch.khash.reserve(hi - lo);
      ch.raw.reserve(hi - lo);
      ch.rawn.reserve(hi - lo);
      Dec dtmp;
      std::string tmp;
      for (uint64_t i = lo; i < hi; ++i) {
        if (ts) ts[i] = rec_ts ? rec_ts[i] : 0;
        st[i] = (uint8_t)decode_one(*dec, buf + off[i], (size_t)(off[i + 1] - off[i]), i, cols, valid, ch, dtmp, tmp,
                                    spell != nullptr);
      }
      ch.koff.push_back(ch.arena.size());
      if (spell) ch.fof.push_back(ch.forms.size());
    };
    if (T == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 1; t < T; ++t) th.emplace_back(work, t);
      work(0);
      for (auto &x : th) x.join();
    }
    // ids in record order
    uint64_t rej = 0;
    for (int t = 0; t < T; ++t) {
      const Chunk &ch = chunks[(size_t)t];
      const uint64_t lo = n * (uint64_t)t / (uint64_t)T, hi = n * (uint64_t)(t + 1) / (uint64_t)T;
      for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t j = i - lo;
        if (st[i] != HSG_DEC_OK) {
          key_id[i] = HSG_KEY_NONE;
          if (spell) spell[i] = HSG_KEY_NONE;
          for (int c = 0; c < C; ++c) valid[c][i] = 0;
          ++rej;
          continue;
        }
        const char *cb = ch.arena.data() + ch.koff[j];
        const size_t cn = (size_t)(ch.koff[j + 1] - ch.koff[j]);
        const char *fb = spell ? ch.forms.data() + ch.fof[j] : nullptr;
        const size_t fnb = spell ? (size_t)(ch.fof[j + 1] - ch.fof[j]) : 0;
        int64_t f = dict->find(cb, cn, ch.khash[j], nullptr);
        if (f < 0) {
          uint32_t id;
          const int rc = dict->insert(cb, cn, ch.khash[j], ch.raw[j], ch.rawn[j], &id, spell ? fb : nullptr, fnb);
          if (rc != HSG_OK) return rc;
          f = id;
        }
        key_id[i] = (uint32_t)f;
        if (spell) {
          const int rc = dict->spelling((uint32_t)f, fb, fnb, ch.raw[j], ch.rawn[j], &spell[i]);
          if (rc != HSG_OK) return rc;
        }
      }
    }
    if (rejected) *rejected = rej;
    return HSG_OK;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  } catch (...) {
    return HSG_E_INVALID;
  }
}

extern "C" int hsg_decode_json(hsg_decoder *dec, hsg_keydict *dict, uint64_t n, const char *buf, const uint64_t *off,
                               const int64_t *rec_ts, uint32_t *key_id, int64_t *ts, void *const *cols,
                               uint8_t *const *valid, uint8_t *status, uint64_t *rejected, int n_threads) {
  return hsg_decode_json_spelled(dec, dict, n, buf, off, rec_ts, key_id, ts, cols, valid, status, rejected, nullptr,
                                 n_threads);
}

extern "C" int hsg_decode_json_batch(hsg_decoder *dec, hsg_keydict *dict, uint64_t n, const char *buf,
                                     const uint64_t *off, const int64_t *rec_ts, hsg_decode_buffers *bufs,
                                     hsg_batch *out, uint8_t *status, uint64_t *rejected, uint32_t *spell,
                                     int n_threads) {
  if (!dec || !bufs || !out || n > bufs->capacity || !bufs->key_id || !bufs->ts) return HSG_E_INVALID;
  const int C = (int)dec->cols.size();
  if (C > 8 || (C && (!bufs->cols || !bufs->valid))) return HSG_E_INVALID;
  int rc = hsg_decode_json_spelled(dec, dict, n, buf, off, rec_ts, bufs->key_id, bufs->ts, bufs->cols, bufs->valid,
                                   status, rejected, spell, n_threads);
  if (rc != HSG_OK) return rc;
  memset(out, 0, sizeof(*out));
  out->n = n;
  out->mem = HSG_MEM_HOST;
  out->n_cols = C;
  out->key_id = bufs->key_id;
  out->ts = bufs->ts;
  int32_t types[8] = {};
  for (int c = 0; c < C; ++c) {
    bufs->col_ptrs[c] = bufs->cols[c];
    bufs->valid_ptrs[c] = bufs->valid[c];
    types[c] = dec->cols[c].type;
  }
  out->cols = bufs->col_ptrs;
  out->valid = bufs->valid_ptrs;
  uint32_t present = 0;
  rc = hsg_batch_narrow(out, types, bufs->allow, bufs->ts_frames, &present, n_threads);
  if (rc != HSG_OK) return rc;
  for (int c = 0; c < C; ++c)
    if ((present >> c) & 1u) bufs->valid_ptrs[c] = nullptr;
  return HSG_OK;
}

extern "C" int hsg_keydict_spelling_text(const hsg_keydict *d, uint32_t spell, char *buf, size_t cap, size_t *len) {
  if (!d || !len) return HSG_E_INVALID;
  if (!(spell & HSG_SPELL_ALT)) return hsg_keydict_text(d, spell, buf, cap, len);
  const uint32_t ix = spell & ~HSG_SPELL_ALT;
  if (ix + 1 >= d->alt_off.size()) return HSG_E_INVALID;
  const uint64_t a = d->alt_off[ix], b = d->alt_off[ix + 1];
  *len = (size_t)(b - a);
  if (cap < *len || (!buf && *len)) return HSG_E_CAPACITY;
  if (*len) memcpy(buf, d->alt_text.data() + a, *len);
  return HSG_OK;
}

namespace hsg {
// For the sink encoder (sink.cpp): the alternate spellings' texts, index after index.
void keydict_alt_texts(const hsg_keydict *d, const char **text, const uint64_t **off, uint64_t *n) {
  *text = d->alt_text.data();
  *off = d->alt_off.data();
  *n = d->alt_off.size() - 1;
}
// For the sink encoder (sink.cpp): the key texts, id after id.
void keydict_texts(const hsg_keydict *d, const char **text, const uint64_t **off, uint64_t *n) {
  *text = d->text.data();
  *off = d->toff.data();
  *n = d->size();
}
}  // namespace hsg
