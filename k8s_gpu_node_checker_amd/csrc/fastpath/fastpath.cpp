// Native CPU hot path of the checker (CPython extension `_fastpath`).
//
// scan_nodelist(buf, result, keys, use_allocatable, want_extras, health_key, NodeExtras,
//               health_condition="", annotation_mode=2)
//   One pass over a kube-apiserver NodeList JSON page.  Only the fields the
//   checker consumes are materialised as Python objects (metadata.name,
//   metadata.labels, one annotation, spec.taints, spec.unschedulable,
//   status.capacity / status.allocatable GPU keys, status.conditions Ready);
//   everything else (images, managedFields, nodeInfo, addresses, ...) is
//   skipped at byte level.  Semantics are those of the pure-Python path
//   (models/node.py), which reproduces reference check-gpu-node.py:172-226:
//   capacity values go through str() and Python int() (zeros kept, "1k"
//   dropped), Ready = a condition with type "Ready" and status "True",
//   duplicate JSON keys: last one wins (as json.loads).  Any shape this code
//   does not model raises FallbackError *before* `result` is touched, and
//   the caller re-scans the page with json.loads.
//
// dumps_indent2(obj)
//   Byte-identical json.dumps(obj, ensure_ascii=False, indent=2) for
//   dict/list/tuple/str/int/bool/None/float trees.  CPython's indent encoder
//   is the pure-Python _make_iterencode, the dominant render cost at 1000
//   nodes (reference check-gpu-node.py:279).
//
// loads(data)
//   json.loads for the per-node health-report annotation (see its comment below); anything it cannot
//   prove identical raises FallbackError and json.loads runs instead.
//
// Known, documented divergence: bytes inside *skipped* string values are not
// UTF-8-validated (json.loads would reject invalid UTF-8 anywhere).

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <immintrin.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <new>
#include <vector>

namespace {

PyObject* g_fallback = nullptr;  // FallbackError
PyObject *k_name, *k_ready, *k_gpus, *k_breakdown, *k_labels, *k_taints, *k_key, *k_value, *k_effect;
PyObject *a_gpu_nodes, *a_ready_gpu_nodes, *a_extras, *a_items_seen;

struct Fallback {
  const char* why;
};

// ---------------------------------------------------------------- scanning --
struct Cursor {
  const char* p;
  const char* end;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  char peek() {
    ws();
    if (p >= end) throw Fallback{"unexpected end"};
    return *p;
  }
  void expect(char c) {
    if (peek() != c) throw Fallback{"unexpected character"};
    ++p;
  }
  bool consume(char c) {
    if (peek() == c) {
      ++p;
      return true;
    }
    return false;
  }
};

// A raw JSON string token: [b, e) excludes the quotes; `esc` if it has backslashes.
struct RawStr {
  const char* b;
  const char* e;
  bool esc;
};

// First '"' or '\\' at or after p (SSE2, 16 bytes per step); e if none.
inline const char* find_quote_or_backslash(const char* p, const char* e) {
  const __m128i q = _mm_set1_epi8('"'), b = _mm_set1_epi8('\\');
  while (e - p >= 16) {
    __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    unsigned m = static_cast<unsigned>(_mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, b))));
    if (m) return p + __builtin_ctz(m);
    p += 16;
  }
  while (p < e && *p != '"' && *p != '\\') ++p;
  return p;
}

// Closing quote of a string whose first backslash is at p (nullptr if unterminated); defined below.
const char* finish_escaped_string(const char* p, const char* e);

RawStr read_raw_string(Cursor& c) {
  c.expect('"');
  const char* b = c.p;
  const char* p = find_quote_or_backslash(b, c.end);
  if (p >= c.end) throw Fallback{"unterminated string"};
  if (*p == '"') {  // the common case: no escapes
    c.p = p + 1;
    return RawStr{b, p, false};
  }
  // Escaped: JSON stored in a string (the agent's health-report annotation) has a backslash every few
  // bytes, so the rest is scanned 64 bytes per step with the escaped-quote mask instead of stopping at
  // every backslash.
  p = finish_escaped_string(p, c.end);
  if (!p) throw Fallback{"unterminated string"};
  c.p = p + 1;
  return RawStr{b, p, true};
}

void append_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}

uint32_t read_u4(const char*& p, const char* e) {
  if (e - p < 4) throw Fallback{"short \\u escape"};
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) {
    int h = hexval(p[i]);
    if (h < 0) throw Fallback{"bad \\u escape"};
    v = (v << 4) | static_cast<uint32_t>(h);
  }
  p += 4;
  return v;
}

// Decoded UTF-8 bytes of a JSON string token.
void decode_into(const RawStr& s, std::string& out) {
  out.clear();
  if (!s.esc) {
    out.assign(s.b, s.e);
    return;
  }
  const char* p = s.b;
  while (p < s.e) {
    char ch = *p++;
    if (ch != '\\') {
      out.push_back(ch);
      continue;
    }
    if (p >= s.e) throw Fallback{"dangling escape"};
    char x = *p++;
    switch (x) {
      case '"': out.push_back('"'); break;
      case '\\': out.push_back('\\'); break;
      case '/': out.push_back('/'); break;
      case 'b': out.push_back('\b'); break;
      case 'f': out.push_back('\f'); break;
      case 'n': out.push_back('\n'); break;
      case 'r': out.push_back('\r'); break;
      case 't': out.push_back('\t'); break;
      case 'u': {
        uint32_t cp = read_u4(p, s.e);
        if (cp >= 0xD800 && cp <= 0xDBFF) {
          if (s.e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* q = p + 2;
            uint32_t lo = read_u4(q, s.e);
            if (lo >= 0xDC00 && lo <= 0xDFFF) {
              p = q;
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              throw Fallback{"lone surrogate"};
            }
          } else {
            throw Fallback{"lone surrogate"};
          }
        } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
          throw Fallback{"lone surrogate"};
        }
        append_utf8(out, cp);
        break;
      }
      default:
        throw Fallback{"bad escape"};
    }
  }
}

bool raw_equals(const RawStr& s, const char* lit, std::string& scratch) {
  size_t n = strlen(lit);
  if (!s.esc) return static_cast<size_t>(s.e - s.b) == n && memcmp(s.b, lit, n) == 0;
  decode_into(s, scratch);
  return scratch.size() == n && memcmp(scratch.data(), lit, n) == 0;
}

PyObject* make_str(const RawStr& s, std::string& scratch) {
  PyObject* o;
  if (!s.esc) {
    o = PyUnicode_DecodeUTF8(s.b, s.e - s.b, "strict");
  } else {
    decode_into(s, scratch);
    o = PyUnicode_DecodeUTF8(scratch.data(), static_cast<Py_ssize_t>(scratch.size()), "strict");
  }
  if (!o) {
    PyErr_Clear();
    throw Fallback{"invalid utf-8"};
  }
  return o;
}

// Per-page cache of the Python str objects made from short, escape-free tokens.  Label keys and most
// label values repeat on every node of a cluster ("kubernetes.io/arch": "amd64", ...): the first node
// creates them, the others share them (one INCREF instead of UTF-8 decode + allocation, and dict
// insertion reuses the cached hash).  Keys point into the page buffer, alive for the whole call.
class StrCache {
 public:
  // sized for the page: ~30 shared strings plus a few unique ones per node, at most half full
  explicit StrCache(size_t items) {
    size_t want = 2 * (32 + 4 * items), n = 64;
    while (n < want && n < kMaxSlots) n <<= 1;
    mask_ = n - 1;
    slots_.resize(n);
  }
  StrCache(const StrCache&) = delete;
  StrCache& operator=(const StrCache&) = delete;
  ~StrCache() {
    for (Slot& e : slots_) Py_XDECREF(e.obj);
  }
  // new reference
  PyObject* get(const RawStr& s, std::string& scratch) {
    const size_t n = static_cast<size_t>(s.e - s.b);
    if (s.esc || n > kMaxLen) return make_str(s, scratch);
    uint64_t h = 1469598103934665603ULL;  // FNV-1a
    for (size_t i = 0; i < n; ++i) h = (h ^ static_cast<unsigned char>(s.b[i])) * 1099511628211ULL;
    size_t i = static_cast<size_t>(h) & mask_;
    for (;;) {
      Slot& e = slots_[i];
      if (!e.obj) break;
      if (e.hash == h && e.len == n && memcmp(e.b, s.b, n) == 0) {
        Py_INCREF(e.obj);
        return e.obj;
      }
      i = (i + 1) & mask_;
    }
    PyObject* o = make_str(s, scratch);
    if (used_ < (mask_ + 1) / 2) {
      Slot& e = slots_[i];
      e.hash = h;
      e.b = s.b;
      e.len = n;
      e.obj = o;
      Py_INCREF(o);
      ++used_;
    }
    return o;
  }

 private:
  static constexpr size_t kMaxSlots = 4096, kMaxLen = 96;
  struct Slot {
    uint64_t hash = 0;
    const char* b = nullptr;
    size_t len = 0;
    PyObject* obj = nullptr;
  };
  std::vector<Slot> slots_;
  size_t mask_ = 0;
  size_t used_ = 0;
};

void skip_value(Cursor& c);

void skip_number(Cursor& c) {
  const char* p = c.p;
  const char* e = c.end;
  if (p < e && *p == '-') ++p;
  if (e - p >= 8 && memcmp(p, "Infinity", 8) == 0) {
    c.p = p + 8;
    return;
  }
  const char* start = p;
  while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) ++p;
  if (p == start) throw Fallback{"bad number"};
  c.p = p;
}

void skip_literal(Cursor& c) {
  const char* p = c.p;
  size_t left = static_cast<size_t>(c.end - p);
  if (left >= 4 && (memcmp(p, "true", 4) == 0 || memcmp(p, "null", 4) == 0)) {
    c.p += 4;
  } else if (left >= 5 && memcmp(p, "false", 5) == 0) {
    c.p += 5;
  } else if (left >= 3 && memcmp(p, "NaN", 3) == 0) {
    c.p += 3;
  } else if (left >= 8 && memcmp(p, "Infinity", 8) == 0) {  // json.loads accepts it too
    c.p += 8;
  } else {
    throw Fallback{"bad literal"};
  }
}

// Skip a whole object/array with a flat bracket counter (string-aware), 16 bytes per step:
// only '"', '{', '}', '[' and ']' stop the vector scan; strings are jumped over whole.
const char* skip_container_sse2(const char* p, const char* e) {
  int depth = 0;
  const __m128i vq = _mm_set1_epi8('"'), vo = _mm_set1_epi8('{'), vc = _mm_set1_epi8('}');
  const __m128i vl = _mm_set1_epi8('['), vr = _mm_set1_epi8(']');
  while (p < e) {
    const char* hit;
    if (e - p >= 16) {
      __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
      __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, vq), _mm_cmpeq_epi8(v, vo)),
                               _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, vc), _mm_cmpeq_epi8(v, vl)),
                                            _mm_cmpeq_epi8(v, vr)));
      unsigned bits = static_cast<unsigned>(_mm_movemask_epi8(m));
      if (!bits) {
        p += 16;
        continue;
      }
      hit = p + __builtin_ctz(bits);
    } else {
      hit = p;
      while (hit < e && *hit != '"' && *hit != '{' && *hit != '}' && *hit != '[' && *hit != ']') ++hit;
      if (hit >= e) break;
    }
    const char ch = *hit;
    if (ch == '"') {
      Cursor t{hit, e};
      read_raw_string(t);
      p = t.p;
      continue;
    }
    if (ch == '{' || ch == '[') {
      ++depth;
    } else if (--depth == 0) {
      return hit + 1;
    }
    p = hit + 1;
  }
  return nullptr;
}

// 64 bytes per step, branch-free string tracking (the simdjson stage-1 idea, written for this
// scanner): backslash runs -> escaped characters, unescaped quotes -> in-string mask via a carry-less
// prefix XOR, then only brackets outside strings are counted.  AVX2 + PCLMUL (runtime-dispatched).
__attribute__((target("avx2,pclmul,popcnt,bmi")))
inline uint64_t eq_mask64(const __m256i lo, const __m256i hi, char ch) {
  const __m256i v = _mm256_set1_epi8(ch);
  const uint32_t a = static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(lo, v)));
  const uint32_t b = static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(hi, v)));
  return static_cast<uint64_t>(a) | (static_cast<uint64_t>(b) << 32);
}

__attribute__((target("avx2,pclmul,popcnt,bmi")))
const char* skip_container_avx2(const char* p, const char* e) {
  int64_t depth = 0;
  uint64_t prev_escaped = 0, prev_in_string = 0;
  const uint64_t even = 0x5555555555555555ULL;
  alignas(32) char tail[64];
  for (const char* base = p; base < e; base += 64) {
    const char* src = base;
    if (e - base < 64) {
      memset(tail, ' ', sizeof tail);
      memcpy(tail, base, static_cast<size_t>(e - base));
      src = tail;
    }
    const __m256i lo = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src));
    const __m256i hi = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + 32));
    uint64_t bs = eq_mask64(lo, hi, '\\');
    uint64_t quotes = eq_mask64(lo, hi, '"');
    // characters escaped by an odd-length backslash run
    bs &= ~prev_escaped;
    const uint64_t follows = (bs << 1) | prev_escaped;
    const uint64_t odd_starts = bs & ~even & ~follows;
    uint64_t even_starts;
    prev_escaped = __builtin_add_overflow(odd_starts, bs, &even_starts) ? 1 : 0;
    const uint64_t escaped = (even ^ (even_starts << 1)) & follows;
    quotes &= ~escaped;
    const uint64_t in_str =
        static_cast<uint64_t>(_mm_cvtsi128_si64(_mm_clmulepi64_si128(_mm_set_epi64x(0, static_cast<long long>(quotes)),
                                                                     _mm_set1_epi8(static_cast<char>(0xFF)), 0))) ^
        prev_in_string;
    prev_in_string = static_cast<uint64_t>(static_cast<int64_t>(in_str) >> 63);
    const uint64_t opens = (eq_mask64(lo, hi, '{') | eq_mask64(lo, hi, '[')) & ~in_str;
    const uint64_t closes = (eq_mask64(lo, hi, '}') | eq_mask64(lo, hi, ']')) & ~in_str;
    const int nc = __builtin_popcountll(closes);
    if (depth > nc) {  // cannot reach depth 0 inside this block
      depth += __builtin_popcountll(opens) - nc;
      continue;
    }
    uint64_t st = opens | closes;
    while (st) {
      const int i = __builtin_ctzll(st);
      if ((opens >> i) & 1) {
        ++depth;
      } else if (--depth == 0) {
        const char* hit = base + i;
        return hit < e ? hit + 1 : nullptr;
      }
      st &= st - 1;
    }
  }
  return nullptr;
}

const bool g_have_avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("pclmul") &&
                         __builtin_cpu_supports("popcnt") && __builtin_cpu_supports("bmi");

__attribute__((target("avx2,pclmul,popcnt,bmi")))
const char* finish_escaped_string_avx2(const char* p, const char* e) {
  // p is a backslash not preceded by one, so no escape carries in
  uint64_t prev_escaped = 0;
  const uint64_t even = 0x5555555555555555ULL;
  alignas(32) char tail[64];
  for (const char* base = p; base < e; base += 64) {
    const char* src = base;
    if (e - base < 64) {
      memset(tail, ' ', sizeof tail);
      memcpy(tail, base, static_cast<size_t>(e - base));
      src = tail;
    }
    const __m256i lo = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src));
    const __m256i hi = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + 32));
    uint64_t bs = eq_mask64(lo, hi, '\\') & ~prev_escaped;
    const uint64_t follows = (bs << 1) | prev_escaped;
    const uint64_t odd_starts = bs & ~even & ~follows;
    uint64_t even_starts;
    prev_escaped = __builtin_add_overflow(odd_starts, bs, &even_starts) ? 1 : 0;
    const uint64_t escaped = (even ^ (even_starts << 1)) & follows;
    const uint64_t quotes = eq_mask64(lo, hi, '"') & ~escaped;
    if (quotes) {
      const char* q = base + __builtin_ctzll(quotes);
      return q < e ? q : nullptr;
    }
  }
  return nullptr;
}

const char* finish_escaped_string(const char* p, const char* e) {
  if (g_have_avx2) return finish_escaped_string_avx2(p, e);
  for (;;) {  // p is at a backslash: skip it and the escaped character, find the next stop
    p = find_quote_or_backslash(p + 2, e);
    if (p >= e) return nullptr;
    if (*p == '"') return p;
  }
}

void skip_container(Cursor& c) {
  const char* end = g_have_avx2 ? skip_container_avx2(c.p, c.end) : skip_container_sse2(c.p, c.end);
  if (!end) throw Fallback{"unterminated container"};
  c.p = end;
}

void skip_value(Cursor& c) {
  char ch = c.peek();
  if (ch == '"') {
    read_raw_string(c);
  } else if (ch == '{' || ch == '[') {
    skip_container(c);
  } else if (ch == '-' || (ch >= '0' && ch <= '9')) {
    skip_number(c);
  } else {
    skip_literal(c);
  }
}

// Iterate the members of an object; `fn(key, cursor)` must consume the value.
template <class F>
void for_members(Cursor& c, F&& fn) {
  c.expect('{');
  if (c.consume('}')) return;
  for (;;) {
    if (c.peek() != '"') throw Fallback{"expected key"};
    RawStr k = read_raw_string(c);
    c.expect(':');
    fn(k, c);
    if (c.consume(',')) continue;
    c.expect('}');
    return;
  }
}

template <class F>
void for_elements(Cursor& c, F&& fn) {
  c.expect('[');
  if (c.consume(']')) return;
  for (;;) {
    fn(c);
    if (c.consume(',')) continue;
    c.expect(']');
    return;
  }
}

bool is_null(Cursor& c) {
  if (c.peek() == 'n') {
    skip_literal(c);
    return true;
  }
  return false;
}

// RAII holder for an owned PyObject*.
struct Ref {
  PyObject* o = nullptr;
  Ref() = default;
  explicit Ref(PyObject* x) : o(x) {}
  Ref(const Ref&) = delete;
  Ref& operator=(const Ref&) = delete;
  Ref(Ref&& r) noexcept : o(r.o) { r.o = nullptr; }
  Ref& operator=(Ref&& r) noexcept {
    if (this != &r) {
      Py_XDECREF(o);
      o = r.o;
      r.o = nullptr;
    }
    return *this;
  }
  ~Ref() { Py_XDECREF(o); }
  void reset(PyObject* x) {
    Py_XDECREF(o);
    o = x;
  }
  PyObject* release() {
    PyObject* x = o;
    o = nullptr;
    return x;
  }
};

// ---------------------------------------------------------------------------
// Two passes per page:
//   pass 1 (GIL released): walk the bytes, validate the shapes this code models,
//          record spans of the fields the checker needs (NodeRec) -- no Python objects;
//   pass 2 (GIL held): for GPU nodes only, materialise dicts/strings/ints from the spans.
// Pass 1 is most of the byte work, so another thread (the kube client's reader of the
// next page) runs concurrently with it.

enum class QKind : uint8_t { Unset, Str, Num, Other };

// One capacity / allocatable entry as it appeared last (json.loads: last duplicate wins).
struct QRaw {
  QKind kind = QKind::Unset;
  RawStr s{nullptr, nullptr, false};  // Str: the string token; Num: the number text
};

enum class VKind : uint8_t { Absent, Null, Str };
struct SRaw {  // an optional string-or-null field
  VKind kind = VKind::Absent;
  RawStr s{nullptr, nullptr, false};
};

struct Span {
  const char* b = nullptr;
  const char* e = nullptr;
};

struct NodeRec {
  bool is_obj = false;
  bool meta_obj = false;
  SRaw name;
  bool labels_obj = false;  // labels present as an object (possibly empty)
  Span labels;
  bool have_health = false;
  RawStr health_raw{nullptr, nullptr, false};
  bool taints_list = false;
  Span taints;
  bool unschedulable = false;
  bool ready = false;
  bool have_ip = false;
  RawStr ip{nullptr, nullptr, false};
  bool have_hc = false;  // AMDGPUHealthy condition
  SRaw hc_status, hc_reason, hc_message;
  bool hc_have_hb = false;
  double hc_hb = 0.0;
  std::vector<QRaw> cap, alloc;
};

struct Pass1Ctx {
  size_t nkeys;
  const std::vector<std::string>* keys;
  const std::string* health_key;
  const std::string* health_cond;
  std::string scratch;
};

void p1_resource_map(Cursor& c, Pass1Ctx& x, std::vector<QRaw>& out) {
  for (auto& q : out) q = QRaw{};
  if (c.peek() != '{') {
    skip_value(c);
    return;
  }
  std::string kd;
  for_members(c, [&](const RawStr& k, Cursor& cc) {
    const char* kb = k.b;
    size_t kn = static_cast<size_t>(k.e - k.b);
    if (k.esc) {
      decode_into(k, kd);
      kb = kd.data();
      kn = kd.size();
    }
    for (size_t i = 0; i < x.nkeys; ++i) {
      const std::string& key = (*x.keys)[i];
      if (key.size() == kn && memcmp(key.data(), kb, kn) == 0) {
        QRaw& q = out[i];
        char ch = cc.peek();
        if (ch == 'n') {  // null -> key treated as missing
          skip_literal(cc);
          q = QRaw{};
        } else if (ch == '"') {
          q.kind = QKind::Str;
          q.s = read_raw_string(cc);
        } else if (ch == '-' || (ch >= '0' && ch <= '9')) {
          q.kind = QKind::Num;
          const char* b = cc.p;
          skip_number(cc);
          q.s = RawStr{b, cc.p, false};
        } else {
          q.kind = QKind::Other;  // bools, objects, arrays: str() of them never parses as int
          skip_value(cc);
        }
        return;
      }
    }
    skip_value(cc);
  });
}

// validate a labels object: string keys -> string values (else the Python path decides)
void p1_labels(Cursor& c, NodeRec& r) {
  if (is_null(c)) {
    r.labels_obj = false;
    return;
  }
  if (c.peek() != '{') throw Fallback{"labels not an object"};
  const char* b = c.p;
  for_members(c, [&](const RawStr&, Cursor& cc) {
    if (cc.peek() != '"') throw Fallback{"label value not a string"};
    read_raw_string(cc);
  });
  r.labels_obj = true;
  r.labels = Span{b, c.p};
}

SRaw p1_str_or_null(Cursor& c, const char* what) {
  SRaw v;
  if (is_null(c)) {
    v.kind = VKind::Null;
  } else if (c.peek() == '"') {
    v.kind = VKind::Str;
    v.s = read_raw_string(c);
  } else {
    throw Fallback{what};
  }
  return v;
}

void p1_metadata(Cursor& c, Pass1Ctx& x, NodeRec& r) {
  r.name = SRaw{};
  r.labels_obj = false;
  r.have_health = false;
  r.meta_obj = false;
  if (c.peek() != '{') {
    skip_value(c);  // null or a non-object: name "" / labels {} (models/node.py)
    return;
  }
  r.meta_obj = true;
  std::string& scratch = x.scratch;
  for_members(c, [&](const RawStr& k, Cursor& cc) {
    if (raw_equals(k, "name", scratch)) {
      r.name = p1_str_or_null(cc, "name not a string");
    } else if (raw_equals(k, "labels", scratch)) {
      p1_labels(cc, r);
    } else if (raw_equals(k, "annotations", scratch)) {
      r.have_health = false;
      if (cc.peek() != '{') {
        skip_value(cc);
        return;
      }
      for_members(cc, [&](const RawStr& ak, Cursor& c3) {
        if (!x.health_key->empty() && raw_equals(ak, x.health_key->c_str(), scratch)) {
          r.have_health = c3.peek() == '"';
          if (r.have_health) r.health_raw = read_raw_string(c3);
          else skip_value(c3);
        } else {
          skip_value(c3);
        }
      });
    } else {
      skip_value(cc);
    }
  });
}

void p1_spec(Cursor& c, Pass1Ctx& x, NodeRec& r) {
  r.taints_list = false;
  r.unschedulable = false;
  if (c.peek() != '{') {
    skip_value(c);
    return;
  }
  std::string& scratch = x.scratch;
  for_members(c, [&](const RawStr& k, Cursor& cc) {
    if (raw_equals(k, "taints", scratch)) {
      r.taints_list = false;
      if (cc.peek() != '[') {
        skip_value(cc);
        return;
      }
      const char* b = cc.p;
      for_elements(cc, [&](Cursor& c3) {
        if (c3.peek() != '{') {
          skip_value(c3);
          return;
        }
        for_members(c3, [&](const RawStr& fk, Cursor& c4) {
          if (raw_equals(fk, "key", scratch) || raw_equals(fk, "value", scratch) || raw_equals(fk, "effect", scratch))
            p1_str_or_null(c4, "taint field not a string");
          else
            skip_value(c4);
        });
      });
      r.taints_list = true;
      r.taints = Span{b, cc.p};
    } else if (raw_equals(k, "unschedulable", scratch)) {
      char ch = cc.peek();
      if (ch == 't') {
        skip_literal(cc);
        r.unschedulable = true;
      } else if (ch == 'f' || ch == 'n') {
        skip_literal(cc);
        r.unschedulable = false;
      } else {
        throw Fallback{"unschedulable not a bool"};
      }
    } else {
      skip_value(cc);
    }
  });
}

// "YYYY-MM-DDTHH:MM:SSZ" -> epoch seconds (the apiserver's RFC 3339 form); other shapes fall back.
double parse_k8s_time(const RawStr& s) {
  if (s.esc || s.e - s.b != 20) throw Fallback{"unusual timestamp"};
  const char* p = s.b;
  auto num = [&](int off, int n) {
    int v = 0;
    for (int i = 0; i < n; ++i) {
      char ch = p[off + i];
      if (ch < '0' || ch > '9') throw Fallback{"unusual timestamp"};
      v = v * 10 + (ch - '0');
    }
    return v;
  };
  if (p[4] != '-' || p[7] != '-' || p[10] != 'T' || p[13] != ':' || p[16] != ':' || p[19] != 'Z')
    throw Fallback{"unusual timestamp"};
  int y = num(0, 4), m = num(5, 2), d = num(8, 2), hh = num(11, 2), mm = num(14, 2), ss = num(17, 2);
  if (m < 1 || m > 12 || d < 1 || d > 31 || hh > 23 || mm > 59 || ss > 59) throw Fallback{"unusual timestamp"};
  // days_from_civil (Howard Hinnant)
  y -= m <= 2;
  const long era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = static_cast<unsigned>(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  const long days = era * 146097 + static_cast<long>(doe) - 719468;
  return static_cast<double>(days) * 86400.0 + hh * 3600.0 + mm * 60.0 + ss;
}

void p1_status(Cursor& c, Pass1Ctx& x, NodeRec& r) {
  for (auto* v : {&r.cap, &r.alloc})
    for (auto& q : *v) q = QRaw{};
  r.ready = false;
  r.have_ip = false;
  r.have_hc = false;
  if (c.peek() != '{') {
    skip_value(c);
    return;
  }
  std::string& scratch = x.scratch;
  for_members(c, [&](const RawStr& k, Cursor& cc) {
    if (raw_equals(k, "capacity", scratch)) {
      p1_resource_map(cc, x, r.cap);
    } else if (raw_equals(k, "allocatable", scratch)) {
      p1_resource_map(cc, x, r.alloc);
    } else if (raw_equals(k, "addresses", scratch)) {
      r.have_ip = false;
      if (cc.peek() != '[') {
        skip_value(cc);
        return;
      }
      for_elements(cc, [&](Cursor& c3) {
        if (c3.peek() != '{') {
          skip_value(c3);
          return;
        }
        bool internal = false, have_addr = false;
        RawStr addr{nullptr, nullptr, false};
        for_members(c3, [&](const RawStr& fk, Cursor& c4) {
          if (raw_equals(fk, "type", scratch) && c4.peek() == '"') {
            internal = raw_equals(read_raw_string(c4), "InternalIP", scratch);
          } else if (raw_equals(fk, "address", scratch) && c4.peek() == '"') {
            addr = read_raw_string(c4);
            have_addr = true;
          } else {
            if (raw_equals(fk, "type", scratch)) internal = false;
            if (raw_equals(fk, "address", scratch)) have_addr = false;
            skip_value(c4);
          }
        });
        if (internal && have_addr && !r.have_ip) {
          r.have_ip = true;
          r.ip = addr;
        }
      });
    } else if (raw_equals(k, "conditions", scratch)) {
      r.ready = false;
      r.have_hc = false;
      if (cc.peek() != '[') {
        skip_value(cc);
        return;
      }
      for_elements(cc, [&](Cursor& c3) {
        if (c3.peek() != '{') {
          skip_value(c3);
          return;
        }
        bool type_ready = false, status_true = false, type_health = false, status_bad = false;
        SRaw st, reason, message;
        st.kind = VKind::Null;
        reason.kind = VKind::Null;
        message.kind = VKind::Null;
        bool have_hb = false;
        double hb = 0.0;
        for_members(c3, [&](const RawStr& fk, Cursor& c4) {
          bool is_type = raw_equals(fk, "type", scratch);
          bool is_status = !is_type && raw_equals(fk, "status", scratch);
          if (is_type) {
            type_ready = type_health = false;
            if (c4.peek() == '"') {
              RawStr v = read_raw_string(c4);
              type_ready = raw_equals(v, "Ready", scratch);
              type_health = !x.health_cond->empty() && raw_equals(v, x.health_cond->c_str(), scratch);
            } else {
              skip_value(c4);
            }
          } else if (is_status) {
            status_true = false;
            status_bad = false;
            if (c4.peek() == '"') {
              RawStr v = read_raw_string(c4);
              status_true = raw_equals(v, "True", scratch);
              st.kind = VKind::Str;
              st.s = v;
            } else if (is_null(c4)) {
              st.kind = VKind::Null;
            } else {
              status_bad = true;  // non-string status: only matters for the health condition
              skip_value(c4);
            }
          } else if (raw_equals(fk, "reason", scratch)) {
            reason = p1_str_or_null(c4, "condition field not a string");
          } else if (raw_equals(fk, "message", scratch)) {
            message = p1_str_or_null(c4, "condition field not a string");
          } else if (raw_equals(fk, "lastHeartbeatTime", scratch)) {
            have_hb = false;
            if (c4.peek() == '"') {
              hb = parse_k8s_time(read_raw_string(c4));
              have_hb = true;
            } else {
              skip_value(c4);
            }
          } else {
            skip_value(c4);
          }
        });
        if (type_ready && status_true) r.ready = true;
        if (type_health) {
          if (status_bad) throw Fallback{"health condition status not a string"};
          r.have_hc = true;
          r.hc_status = st;
          r.hc_reason = reason;
          r.hc_message = message;
          r.hc_have_hb = have_hb;
          r.hc_hb = hb;
        }
      });
    } else {
      skip_value(cc);
    }
  });
}

void p1_item(Cursor& c, Pass1Ctx& x, NodeRec& r) {
  r.cap.assign(x.nkeys, QRaw{});
  r.alloc.assign(x.nkeys, QRaw{});
  if (c.peek() != '{') {
    skip_value(c);  // non-object item: never a GPU node
    r.is_obj = false;
    return;
  }
  r.is_obj = true;
  std::string& scratch = x.scratch;
  for_members(c, [&](const RawStr& k, Cursor& cc) {
    if (raw_equals(k, "metadata", scratch)) p1_metadata(cc, x, r);
    else if (raw_equals(k, "spec", scratch)) p1_spec(cc, x, r);
    else if (raw_equals(k, "status", scratch)) p1_status(cc, x, r);
    else skip_value(cc);
  });
}

struct Pass1Out {
  std::vector<NodeRec> items;
  bool have_cont = false;
  RawStr cont{nullptr, nullptr, false};
};

// The whole page, no Python API calls (runs with the GIL released).
void pass1(const char* b, const char* e, Pass1Ctx& x, Pass1Out& out) {
  Cursor c{b, e};
  if (c.peek() != '{') throw Fallback{"top level is not an object"};
  bool items_seen = false;
  std::string& scratch = x.scratch;
  for_members(c, [&](const RawStr& k, Cursor& cc) {
    if (raw_equals(k, "items", scratch)) {
      if (items_seen) throw Fallback{"duplicate items"};
      items_seen = true;
      if (is_null(cc)) return;
      if (cc.peek() != '[') throw Fallback{"items not a list"};
      for_elements(cc, [&](Cursor& c3) {
        out.items.emplace_back();
        p1_item(c3, x, out.items.back());
      });
    } else if (raw_equals(k, "metadata", scratch)) {
      out.have_cont = false;
      if (cc.peek() != '{') {
        skip_value(cc);
        return;
      }
      for_members(cc, [&](const RawStr& mk, Cursor& c3) {
        if (raw_equals(mk, "continue", scratch)) {
          out.have_cont = false;
          if (c3.peek() == '"') {
            RawStr v = read_raw_string(c3);
            if (v.e > v.b) {
              out.have_cont = true;
              out.cont = v;
            }
          } else {
            skip_value(c3);
          }
        } else {
          skip_value(c3);
        }
      });
    } else {
      skip_value(cc);
    }
  });
  c.ws();
  if (c.p != c.end) throw Fallback{"trailing data"};
}

// ------------------------------------------------------------ pass 2 (GIL) --
PyObject* parse_int_text(const char* b, size_t n, std::string& scratch) {
  // Fast path: optional sign + ASCII digits, nothing else.
  const char* p = b;
  const char* e = b + n;
  const char* q = p;
  if (q < e && (*q == '+' || *q == '-')) ++q;
  bool simple = q < e && (e - q) <= 18;
  for (const char* r = q; simple && r < e; ++r)
    if (*r < '0' || *r > '9') simple = false;
  if (simple) {
    long long v = 0;
    for (const char* r = q; r < e; ++r) v = v * 10 + (*r - '0');
    if (*p == '-') v = -v;
    return PyLong_FromLongLong(v);
  }
  // Exact Python int(str) semantics (whitespace, '_' separators, unicode digits).
  scratch.assign(b, n);
  PyObject* s = PyUnicode_DecodeUTF8(scratch.data(), static_cast<Py_ssize_t>(scratch.size()), "strict");
  if (!s) {
    PyErr_Clear();
    throw Fallback{"invalid utf-8 in quantity"};
  }
  PyObject* v = PyLong_FromUnicodeObject(s, 10);
  Py_DECREF(s);
  if (!v) {
    if (PyErr_ExceptionMatches(PyExc_ValueError)) {
      PyErr_Clear();
      return nullptr;  // dropped, as the reference's `except Exception: pass`
    }
    PyErr_Clear();
    throw Fallback{"int() raised"};
  }
  return v;
}

// str()+int() semantics of one QRaw; nullptr = not in the breakdown
PyObject* quantity_value(const QRaw& q, std::string& scratch) {
  if (q.kind == QKind::Unset || q.kind == QKind::Other) return nullptr;
  if (q.kind == QKind::Num) {
    size_t n = static_cast<size_t>(q.s.e - q.s.b);
    for (size_t i = 0; i < n; ++i) {
      char ch = q.s.b[i];
      if (ch == '.' || ch == 'e' || ch == 'E' || ch == 'I') return nullptr;  // str(float): never int()-parsable
    }
    return parse_int_text(q.s.b, n, scratch);
  }
  const char* b = q.s.b;
  size_t n = static_cast<size_t>(q.s.e - q.s.b);
  std::string dec;
  if (q.s.esc) {
    decode_into(q.s, dec);
    b = dec.data();
    n = dec.size();
  }
  if (n == 0) return nullptr;  // `if not val: continue`
  return parse_int_text(b, n, scratch);
}

PyObject* breakdown(const std::vector<PyObject*>& pykeys, const std::vector<QRaw>& qs, long long* total,
                    std::string& scratch) {
  PyObject* d = PyDict_New();
  if (!d) throw Fallback{"oom"};
  Ref hold(d);
  long long sum = 0;
  for (size_t i = 0; i < pykeys.size(); ++i) {
    PyObject* v = quantity_value(qs[i], scratch);
    if (!v) continue;
    Ref hv(v);
    if (PyDict_SetItem(d, pykeys[i], v) < 0) throw Fallback{"dict"};
    int of = 0;
    long long x = PyLong_AsLongLongAndOverflow(v, &of);
    if (of) throw Fallback{"huge quantity"};
    sum += x;
  }
  if (total) *total = sum;
  return hold.release();
}

PyObject* sraw_obj(const SRaw& v, std::string& scratch) {
  if (v.kind != VKind::Str) Py_RETURN_NONE;
  return make_str(v.s, scratch);
}

PyObject* sraw_cached(const SRaw& v, StrCache& cache, std::string& scratch) {
  if (v.kind != VKind::Str) Py_RETURN_NONE;
  return cache.get(v.s, scratch);
}

PyObject* labels_dict(const NodeRec& r, StrCache& cache, std::string& scratch) {
  PyObject* d = PyDict_New();
  if (!d) throw Fallback{"oom"};
  Ref hold(d);
  if (!r.labels_obj) return hold.release();
  Cursor c{r.labels.b, r.labels.e};
  for_members(c, [&](const RawStr& k, Cursor& cc) {
    Ref key(cache.get(k, scratch));
    Ref val(cache.get(read_raw_string(cc), scratch));
    if (PyDict_SetItem(d, key.o, val.o) < 0) throw Fallback{"dict"};
  });
  return hold.release();
}

PyObject* taints_list(const NodeRec& r, StrCache& cache, std::string& scratch) {
  PyObject* lst = PyList_New(0);
  if (!lst) throw Fallback{"oom"};
  Ref hold(lst);
  if (!r.taints_list) return hold.release();
  Cursor c{r.taints.b, r.taints.e};
  for_elements(c, [&](Cursor& c3) {
    if (c3.peek() != '{') {
      skip_value(c3);
      return;
    }
    Ref tk(Py_NewRef(Py_None)), tv(Py_NewRef(Py_None)), te(Py_NewRef(Py_None));
    for_members(c3, [&](const RawStr& fk, Cursor& c4) {
      if (raw_equals(fk, "key", scratch)) tk.reset(sraw_cached(p1_str_or_null(c4, "taint"), cache, scratch));
      else if (raw_equals(fk, "value", scratch)) tv.reset(sraw_cached(p1_str_or_null(c4, "taint"), cache, scratch));
      else if (raw_equals(fk, "effect", scratch)) te.reset(sraw_cached(p1_str_or_null(c4, "taint"), cache, scratch));
      else skip_value(c4);
    });
    PyObject* d = PyDict_New();
    if (!d) throw Fallback{"oom"};
    Ref hd(d);
    if (PyDict_SetItem(d, k_key, tk.o) < 0 || PyDict_SetItem(d, k_value, tv.o) < 0 ||
        PyDict_SetItem(d, k_effect, te.o) < 0 || PyList_Append(lst, d) < 0)
      throw Fallback{"dict"};
  });
  return hold.release();
}

struct PageOut {
  Ref gpu_nodes{PyList_New(0)};
  Ref ready_nodes{PyList_New(0)};
  Ref extras{PyList_New(0)};
  Ref cont;  // str or nullptr
  Py_ssize_t items = 0;
};

// NodeExtras (models/node.py: a __slots__ class) built without running its Python __init__: the
// instance is allocated by the type and each slot set through its member descriptor, in __init__'s
// order.  Resolved once per page; anything unexpected (not a type, missing or non-member slot)
// keeps the plain constructor call.
struct ExtrasMaker {
  static constexpr int kN = 7;
  PyObject* cls = nullptr;
  PyObject* descr[kN] = {};
  bool direct = false;

  explicit ExtrasMaker(PyObject* c) : cls(c) {
    static const char* names[kN] = {"ready_condition", "capacity",         "allocatable",     "unschedulable",
                                    "health_annotation", "internal_ip", "health_condition"};
    if (!PyType_Check(c)) return;
    PyTypeObject* t = reinterpret_cast<PyTypeObject*>(c);
    if (t->tp_init == nullptr || t->tp_alloc == nullptr) return;
    for (int i = 0; i < kN; ++i) {
      PyObject* d = PyObject_GetAttrString(c, names[i]);
      if (!d) {
        PyErr_Clear();
        return;
      }
      descr[i] = d;
      if (strcmp(Py_TYPE(d)->tp_name, "member_descriptor") != 0 || Py_TYPE(d)->tp_descr_set == nullptr) return;
    }
    direct = true;
  }
  ExtrasMaker(const ExtrasMaker&) = delete;
  ExtrasMaker& operator=(const ExtrasMaker&) = delete;
  ~ExtrasMaker() {
    for (PyObject* d : descr) Py_XDECREF(d);
  }
  // new reference or nullptr (Python error set)
  PyObject* make(PyObject* const (&vals)[kN]) {
    if (!direct)
      return PyObject_CallFunctionObjArgs(cls, vals[0], vals[1], vals[2], vals[3], vals[4], vals[5], vals[6], nullptr);
    PyTypeObject* t = reinterpret_cast<PyTypeObject*>(cls);
    PyObject* o = t->tp_alloc(t, 0);
    if (!o) return nullptr;
    for (int i = 0; i < kN; ++i) {
      if (Py_TYPE(descr[i])->tp_descr_set(descr[i], o, vals[i]) < 0) {
        Py_DECREF(o);
        return nullptr;
      }
    }
    return o;
  }
};

void emit_node(const NodeRec& r, const std::vector<PyObject*>& pykeys, bool use_alloc, bool want_extras,
               ExtrasMaker& extras, int annot_mode, PageOut& out, StrCache& cache, std::string& scratch) {
  if (!r.is_obj) return;
  long long total = 0;
  Ref bd(breakdown(pykeys, use_alloc ? r.alloc : r.cap, &total, scratch));
  bool ready = r.ready;
  if (total <= 0) {
    // not a GPU node (reference :222) -- unless, counting allocatable, the capacity still registers GPUs:
    // the device plugin withdrew every one, and the node stays in the set as not Ready
    // (models/node.py classify_node)
    if (!use_alloc) return;
    long long cap_total = 0;
    Ref capbd(breakdown(pykeys, r.cap, &cap_total, scratch));
    if (cap_total <= 0) return;
    ready = false;
  }
  PyObject* info = PyDict_New();
  if (!info) throw Fallback{"oom"};
  Ref hi(info);
  Ref name(r.meta_obj ? sraw_obj(r.name, scratch) : PyUnicode_FromStringAndSize("", 0));
  Ref labels(labels_dict(r, cache, scratch));
  Ref taints(taints_list(r, cache, scratch));
  Ref gpus(PyLong_FromLongLong(total));
  if (!name.o || !gpus.o) throw Fallback{"oom"};
  if (PyDict_SetItem(info, k_name, name.o) < 0 || PyDict_SetItem(info, k_ready, ready ? Py_True : Py_False) < 0 ||
      PyDict_SetItem(info, k_gpus, gpus.o) < 0 || PyDict_SetItem(info, k_breakdown, bd.o) < 0 ||
      PyDict_SetItem(info, k_labels, labels.o) < 0 || PyDict_SetItem(info, k_taints, taints.o) < 0)
    throw Fallback{"dict"};
  if (PyList_Append(out.gpu_nodes.o, info) < 0) throw Fallback{"list"};
  if (ready && PyList_Append(out.ready_nodes.o, info) < 0) throw Fallback{"list"};
  if (!want_extras) return;
  Ref capd(breakdown(pykeys, r.cap, nullptr, scratch));
  Ref allocd(breakdown(pykeys, r.alloc, nullptr, scratch));
  Ref hc;
  if (r.have_hc) {
    Ref st(sraw_obj(r.hc_status, scratch)), rs(sraw_obj(r.hc_reason, scratch)), ms(sraw_obj(r.hc_message, scratch));
    Ref hb(r.hc_have_hb ? PyFloat_FromDouble(r.hc_hb) : Py_NewRef(Py_None));
    hc.reset(PyTuple_Pack(4, st.o, rs.o, ms.o, hb.o));
    if (!hc.o) throw Fallback{"oom"};
  }
  // the annotation (full probe report, KBs of escaped JSON) is only materialised when the
  // caller will read it: always (mode 2) or for nodes without the AMDGPUHealthy condition (mode 1)
  Ref health_str;
  if (r.have_health && (annot_mode == 2 || (annot_mode == 1 && !r.have_hc)))
    health_str.reset(make_str(r.health_raw, scratch));
  Ref ip;
  if (r.have_ip) ip.reset(make_str(r.ip, scratch));
  PyObject* const vals[ExtrasMaker::kN] = {r.ready ? Py_True : Py_False,
                                            capd.o,
                                            allocd.o,
                                            r.unschedulable ? Py_True : Py_False,
                                            health_str.o ? health_str.o : Py_None,
                                            ip.o ? ip.o : Py_None,
                                            hc.o ? hc.o : Py_None};
  Ref ex(extras.make(vals));
  if (!ex.o) {
    PyErr_Clear();
    throw Fallback{"NodeExtras()"};
  }
  if (PyList_Append(out.extras.o, ex.o) < 0) throw Fallback{"list"};
}

int append_all(PyObject* result, PyObject* attr, PyObject* items) {
  PyObject* lst = PyObject_GetAttr(result, attr);
  if (!lst) return -1;
  Py_ssize_t n = PyList_GET_SIZE(items);
  int rc = 0;
  if (PyList_Check(lst)) {
    rc = PyList_SetSlice(lst, PyList_GET_SIZE(lst), PyList_GET_SIZE(lst), items);
  } else {
    for (Py_ssize_t i = 0; i < n && rc == 0; ++i) {
      PyObject* r = PyObject_CallMethod(lst, "append", "O", PyList_GET_ITEM(items, i));
      if (!r) rc = -1;
      Py_XDECREF(r);
    }
  }
  Py_DECREF(lst);
  return rc;
}

// Page-scan state between pass 1 (no GIL, any thread) and pass 2 (GIL): the page's buffer stays
// exported (RawStr pointers point into it) until the state is released.
struct PageScan {
  Py_buffer view{};
  bool have_view = false;
  std::vector<std::string> kstr;
  std::string health_key, health_cond;
  Pass1Ctx ctx{0, nullptr, nullptr, nullptr, {}};
  Pass1Out p1;
  const char* why = nullptr;
  ~PageScan() {
    if (have_view) PyBuffer_Release(&view);
  }
};

// Keys as UTF-8 strings (kstr) plus borrowed references (pykeys); false with a Python error set.
bool read_keys(PyObject* keys, std::vector<std::string>& kstr, std::vector<PyObject*>* pykeys) {
  for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(keys); ++i) {
    PyObject* k = PyTuple_GET_ITEM(keys, i);
    Py_ssize_t n;
    const char* s = PyUnicode_AsUTF8AndSize(k, &n);
    if (!s) return false;
    kstr.emplace_back(s, static_cast<size_t>(n));
    if (pykeys) pykeys->push_back(k);
  }
  return true;
}

// Pass 1 over an exported page; the caller holds (or has released) the GIL as it sees fit.
void run_pass1(PageScan& ps) {
  ps.ctx = Pass1Ctx{ps.kstr.size(), &ps.kstr, &ps.health_key, &ps.health_cond, {}};
  const char* b = static_cast<const char*>(ps.view.buf);
  try {
    pass1(b, b + ps.view.len, ps.ctx, ps.p1);
  } catch (const Fallback& f) {
    ps.why = f.why;
  } catch (const std::bad_alloc&) {
    ps.why = "out of memory";
  }
}

// Pass 2 + commit into `result`; returns (continue, items) or nullptr with an error set.
PyObject* finish_scan(PageScan& ps, PyObject* result, const std::vector<PyObject*>& pykeys, int use_alloc,
                      int want_extras, PyObject* extras_cls, int annot_mode) {
  const char* why = ps.why;
  PageOut out;
  if (!why) {
    try {
      if (!out.gpu_nodes.o || !out.ready_nodes.o || !out.extras.o) throw Fallback{"oom"};
      std::string& scratch = ps.ctx.scratch;
      StrCache cache(ps.p1.items.size());
      ExtrasMaker maker(extras_cls);
      for (const NodeRec& r : ps.p1.items)
        emit_node(r, pykeys, use_alloc, want_extras, maker, annot_mode, out, cache, scratch);
      out.items = static_cast<Py_ssize_t>(ps.p1.items.size());
      if (ps.p1.have_cont) out.cont.reset(make_str(ps.p1.cont, scratch));
    } catch (const Fallback& f) {
      why = f.why;
    }
  }
  if (why) {
    if (!PyErr_Occurred()) PyErr_SetString(g_fallback, why);
    return nullptr;
  }
  // commit: nothing above touched `result`
  if (append_all(result, a_gpu_nodes, out.gpu_nodes.o) < 0 ||
      append_all(result, a_ready_gpu_nodes, out.ready_nodes.o) < 0 ||
      (want_extras && append_all(result, a_extras, out.extras.o) < 0))
    return nullptr;
  PyObject* seen = PyObject_GetAttr(result, a_items_seen);
  if (!seen) return nullptr;
  PyObject* n = PyLong_FromSsize_t(out.items);
  PyObject* tot = n ? PyNumber_Add(seen, n) : nullptr;
  Py_DECREF(seen);
  Py_XDECREF(n);
  if (!tot) return nullptr;
  int rc = PyObject_SetAttr(result, a_items_seen, tot);
  Py_DECREF(tot);
  if (rc < 0) return nullptr;
  PyObject* cont = out.cont.o ? out.cont.o : Py_None;
  return Py_BuildValue("(On)", cont, out.items);
}

PyObject* scan_nodelist(PyObject*, PyObject* args) {
  PageScan ps;
  PyObject *result, *keys, *extras_cls;
  int use_alloc, want_extras;
  const char* health_key_c;
  const char* health_cond_c = "";
  int annot_mode = 2;
  if (!PyArg_ParseTuple(args, "y*OO!ppsO|si", &ps.view, &result, &PyTuple_Type, &keys, &use_alloc, &want_extras,
                        &health_key_c, &extras_cls, &health_cond_c, &annot_mode))
    return nullptr;
  ps.have_view = true;
  std::vector<PyObject*> pykeys;
  if (!read_keys(keys, ps.kstr, &pykeys)) return nullptr;
  ps.health_key = health_key_c;
  ps.health_cond = health_cond_c;
  // pass 1 without the GIL: the buffer is held by `view` (a bytearray cannot be resized while exported)
  Py_BEGIN_ALLOW_THREADS
  run_pass1(ps);
  Py_END_ALLOW_THREADS
  return finish_scan(ps, result, pykeys, use_alloc, want_extras, extras_cls, annot_mode);
}

const char* const kPageScanCapsule = "k8s_gpu_node_checker_amd._fastpath.PageScan";

void page_scan_capsule_free(PyObject* cap) {
  delete static_cast<PageScan*>(PyCapsule_GetPointer(cap, kPageScanCapsule));
}

// Pass 1 only, GIL released: the pipelined page reader runs it on its own thread as soon as a page
// has arrived, so the main thread's pass 2 of the previous page and this page's pass 1 overlap.
// A page pass 1 cannot model is not an error here; scan_prescanned raises FallbackError for it.
PyObject* prescan_nodelist(PyObject*, PyObject* args) {
  auto* ps = new PageScan();
  PyObject* keys;
  const char* health_key_c;
  const char* health_cond_c;
  if (!PyArg_ParseTuple(args, "y*O!ss", &ps->view, &PyTuple_Type, &keys, &health_key_c, &health_cond_c)) {
    delete ps;
    return nullptr;
  }
  ps->have_view = true;
  if (!read_keys(keys, ps->kstr, nullptr)) {
    delete ps;
    return nullptr;
  }
  ps->health_key = health_key_c;
  ps->health_cond = health_cond_c;
  Py_BEGIN_ALLOW_THREADS
  run_pass1(*ps);
  Py_END_ALLOW_THREADS
  PyObject* cap = PyCapsule_New(ps, kPageScanCapsule, page_scan_capsule_free);
  if (!cap) delete ps;
  return cap;
}

// Pass 2 of a prescanned page into `result`; keys must be the ones prescan_nodelist was given.
PyObject* scan_prescanned(PyObject*, PyObject* args) {
  PyObject *cap, *result, *keys, *extras_cls;
  int use_alloc, want_extras;
  int annot_mode = 2;
  if (!PyArg_ParseTuple(args, "OOO!ppO|i", &cap, &result, &PyTuple_Type, &keys, &use_alloc, &want_extras,
                        &extras_cls, &annot_mode))
    return nullptr;
  auto* ps = static_cast<PageScan*>(PyCapsule_GetPointer(cap, kPageScanCapsule));
  if (!ps) return nullptr;
  std::vector<std::string> kstr;
  std::vector<PyObject*> pykeys;
  if (!read_keys(keys, kstr, &pykeys)) return nullptr;
  if (kstr != ps->kstr) {
    PyErr_SetString(PyExc_ValueError, "keys differ from the prescan's");
    return nullptr;
  }
  return finish_scan(*ps, result, pykeys, use_alloc, want_extras, extras_cls, annot_mode);
}

// ---------------------------------------------------------------- emitting --
// The report is mostly ASCII keys, names and label values, ~40 short strings a node.  The output goes to a raw
// growable buffer with one capacity check per string (worst case 6 bytes a byte, all \u00XX) instead of a
// std::string append per piece; strings are copied 16 bytes at a time until a byte that needs an escape (< 0x20,
// '"', '\\'); ints below 2^63 are formatted without a Python object; an all-ASCII document becomes a str by one
// memcpy (no UTF-8 decode pass).
struct Emitter {
  char* base = nullptr;
  char* p = nullptr;
  char* end = nullptr;
  bool ascii = true;  // every byte so far < 0x80: the result is built as a 1-byte-kind str
  Emitter() = default;
  Emitter(const Emitter&) = delete;
  Emitter& operator=(const Emitter&) = delete;
  ~Emitter() { std::free(base); }
  void reserve(size_t extra) {
    if (static_cast<size_t>(end - p) >= extra) return;
    const size_t used = static_cast<size_t>(p - base);
    size_t cap = static_cast<size_t>(end - base);
    cap = cap ? cap : 4096;
    while (cap - used < extra) cap *= 2;
    char* nb = static_cast<char*>(std::realloc(base, cap));
    if (!nb) throw std::bad_alloc();
    base = nb;
    p = nb + used;
    end = nb + cap;
  }
  void put(const char* s, size_t n) {  // after reserve()
    std::memcpy(p, s, n);
    p += n;
  }
  void append(const char* s, size_t n) {
    reserve(n);
    put(s, n);
  }
  size_t size() const { return static_cast<size_t>(p - base); }
};

// First byte at or after p that a JSON string must escape, e if none; *high |= any byte >= 0x80 before it.
inline const char* find_escape(const char* p, const char* e, bool* high) {
  const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), lim = _mm_set1_epi8(0x1F);
  __m128i hi = _mm_setzero_si128();
  while (e - p >= 16) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    const __m128i ctl = _mm_cmpeq_epi8(_mm_min_epu8(v, lim), v);  // unsigned v <= 0x1F
    const unsigned m = static_cast<unsigned>(
        _mm_movemask_epi8(_mm_or_si128(ctl, _mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, bs)))));
    if (m) {
      const int k = __builtin_ctz(m);
      // the bytes before the escape: high bit set on any of them?
      if ((static_cast<unsigned>(_mm_movemask_epi8(v)) & ((1u << k) - 1u)) || _mm_movemask_epi8(hi)) *high = true;
      return p + k;
    }
    hi = _mm_or_si128(hi, v);
    p += 16;
  }
  if (_mm_movemask_epi8(hi)) *high = true;
  for (; p < e; ++p) {
    const unsigned char ch = static_cast<unsigned char>(*p);
    if (ch < 0x20 || ch == '"' || ch == '\\') return p;
    if (ch >= 0x80) *high = true;
  }
  return e;
}

constexpr int kIndentMax = 64;  // levels served from the run below; deeper ones write spaces
const char kIndentRun[] =
    "\n                                                                                                    "
    "                            ";

// Reserves `extra` more bytes than the indent itself needs.
inline void emit_indent(Emitter& em, int level, size_t extra = 0) {
  const size_t n = 1 + 2 * static_cast<size_t>(level);
  em.reserve(n + extra);
  if (level <= kIndentMax) {
    em.put(kIndentRun, n);
  } else {
    *em.p++ = '\n';
    std::memset(em.p, ' ', n - 1);
    em.p += n - 1;
  }
}

void emit_string(Emitter& em, PyObject* s) {
  Py_ssize_t n;
  const char* u;
  if (PyUnicode_IS_COMPACT_ASCII(s)) {  // the common case: the str's own bytes are its UTF-8
    u = static_cast<const char*>(PyUnicode_DATA(s));
    n = PyUnicode_GET_LENGTH(s);
  } else {
    u = PyUnicode_AsUTF8AndSize(s, &n);
    if (!u) {
      PyErr_Clear();
      throw Fallback{"unencodable string"};
    }
  }
  em.reserve(6 * static_cast<size_t>(n) + 4);  // every byte escaped as \u00XX, the quotes, ": "
  *em.p++ = '"';
  const char* p = u;
  const char* e = u + n;
  static const char hex[] = "0123456789abcdef";
  for (;;) {
    bool high = false;
    const char* q = find_escape(p, e, &high);
    if (high) em.ascii = false;
    em.put(p, static_cast<size_t>(q - p));
    if (q == e) break;
    const unsigned char ch = static_cast<unsigned char>(*q);
    char* o = em.p;
    switch (ch) {
      case '"': o[0] = '\\'; o[1] = '"'; em.p += 2; break;
      case '\\': o[0] = '\\'; o[1] = '\\'; em.p += 2; break;
      case '\n': o[0] = '\\'; o[1] = 'n'; em.p += 2; break;
      case '\r': o[0] = '\\'; o[1] = 'r'; em.p += 2; break;
      case '\t': o[0] = '\\'; o[1] = 't'; em.p += 2; break;
      case '\b': o[0] = '\\'; o[1] = 'b'; em.p += 2; break;
      case '\f': o[0] = '\\'; o[1] = 'f'; em.p += 2; break;
      default: {
        const char buf[6] = {'\\', 'u', '0', '0', hex[ch >> 4], hex[ch & 15]};
        em.put(buf, 6);
      }
    }
    p = q + 1;
  }
  *em.p++ = '"';
}

void emit_float(Emitter& em, PyObject* o) {
  double d = PyFloat_AS_DOUBLE(o);
  if (std::isnan(d)) {
    em.append("NaN", 3);
  } else if (std::isinf(d)) {
    if (d > 0)
      em.append("Infinity", 8);
    else
      em.append("-Infinity", 9);
  } else {
    PyObject* r = PyObject_Repr(o);
    if (!r) throw Fallback{"repr"};
    Py_ssize_t n;
    const char* u = PyUnicode_AsUTF8AndSize(r, &n);
    em.append(u, static_cast<size_t>(n));
    Py_DECREF(r);
  }
}

void emit_int(Emitter& em, PyObject* o) {
  int overflow = 0;
  const long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
  if (!overflow && !(v == -1 && PyErr_Occurred())) {
    char buf[24];
    char* q = buf + sizeof buf;
    unsigned long long m = v < 0 ? 0ULL - static_cast<unsigned long long>(v) : static_cast<unsigned long long>(v);
    do {
      *--q = static_cast<char>('0' + m % 10);
      m /= 10;
    } while (m);
    if (v < 0) *--q = '-';
    em.append(q, static_cast<size_t>(buf + sizeof buf - q));
    return;
  }
  PyErr_Clear();
  PyObject* r = PyObject_Str(o);  // beyond 64 bits: int.__str__ (CPython's own digit limit applies)
  if (!r) throw Fallback{"str"};
  Py_ssize_t n;
  const char* u = PyUnicode_AsUTF8AndSize(r, &n);
  em.append(u, static_cast<size_t>(n));
  Py_DECREF(r);
}

void emit_value(Emitter& em, PyObject* o, int level) {
  if (level > 200) throw Fallback{"too deep"};
  if (o == Py_None) {
    em.append("null", 4);
  } else if (o == Py_True) {
    em.append("true", 4);
  } else if (o == Py_False) {
    em.append("false", 5);
  } else if (PyUnicode_CheckExact(o)) {
    emit_string(em, o);
  } else if (PyLong_CheckExact(o)) {
    emit_int(em, o);
  } else if (PyFloat_CheckExact(o)) {
    emit_float(em, o);
  } else if (PyDict_CheckExact(o)) {
    if (PyDict_GET_SIZE(o) == 0) {
      em.append("{}", 2);
      return;
    }
    em.append("{", 1);
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    bool first = true;
    while (PyDict_Next(o, &pos, &k, &v)) {
      if (!PyUnicode_CheckExact(k)) throw Fallback{"non-str key"};
      if (!first) em.append(",", 1);
      first = false;
      emit_indent(em, level + 1);
      emit_string(em, k);  // reserved room for the ": " after it
      em.put(": ", 2);
      emit_value(em, v, level + 1);
    }
    emit_indent(em, level, 1);
    *em.p++ = '}';
  } else if (PyList_CheckExact(o) || PyTuple_CheckExact(o)) {
    PyObject* seq = o;
    Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n == 0) {
      em.append("[]", 2);
      return;
    }
    em.append("[", 1);
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) em.append(",", 1);
      emit_indent(em, level + 1);
      emit_value(em, PySequence_Fast_GET_ITEM(seq, i), level + 1);
    }
    emit_indent(em, level, 1);
    *em.p++ = ']';
  } else {
    throw Fallback{"unsupported type"};
  }
}

PyObject* dumps_indent2(PyObject*, PyObject* obj) {
  Emitter em;
  try {
    em.reserve(1 << 16);
    emit_value(em, obj, 0);
  } catch (const Fallback& f) {
    if (!PyErr_Occurred()) PyErr_SetString(g_fallback, f.why);
    return nullptr;
  } catch (const std::bad_alloc&) {
    return PyErr_NoMemory();
  }
  const Py_ssize_t n = static_cast<Py_ssize_t>(em.size());
  if (em.ascii) {
    PyObject* s = PyUnicode_New(n, 127);
    if (s) std::memcpy(PyUnicode_1BYTE_DATA(s), em.base, static_cast<size_t>(n));
    return s;
  }
  return PyUnicode_DecodeUTF8(em.base, n, "surrogatepass");
}

// ------------------------------------------------------------------ loads --
// loads(data: bytes | bytearray | str) -> object: json.loads for documents this parser can prove it
// reads the same way (RFC 8259 grammar plus Python's NaN / Infinity / -Infinity, duplicate keys: last
// value at the first key's position, ints of any size via int(), floats via float()).  Anything else
// -- a syntax error, a raw control character in a string, invalid UTF-8, a lone surrogate escape, a
// BOM, nesting deeper than kMaxDepth -- raises FallbackError and the caller re-parses with json.loads,
// which then raises (or succeeds) exactly as it always would.  Used for the agent's health-report
// annotation on every node, so a cold `check-gpu-node` never imports the json package.
constexpr int kMaxDepth = 256;

bool has_control(const char* b, const char* e) {
  const __m128i lim = _mm_set1_epi8(0x1F);
  while (e - b >= 16) {
    __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(b));
    // unsigned v <= 0x1F  <=>  min(v, 0x1F) == v
    if (_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_min_epu8(v, lim), v))) return true;
    b += 16;
  }
  for (; b < e; ++b)
    if (static_cast<unsigned char>(*b) < 0x20) return true;
  return false;
}

PyObject* loads_string(Cursor& c, std::string& scratch) {
  RawStr s = read_raw_string(c);
  if (has_control(s.b, s.e)) throw Fallback{"control character in string"};
  return make_str(s, scratch);
}

PyObject* loads_number(Cursor& c, std::string& scratch) {
  const char* b = c.p;
  const char* p = b;
  const char* e = c.end;
  if (p < e && *p == '-') {
    ++p;
    if (e - p >= 8 && memcmp(p, "Infinity", 8) == 0) {
      c.p = p + 8;
      return PyFloat_FromDouble(-HUGE_VAL);
    }
  }
  if (p >= e) throw Fallback{"bad number"};
  if (*p == '0') {
    ++p;
  } else if (*p >= '1' && *p <= '9') {
    while (p < e && *p >= '0' && *p <= '9') ++p;
  } else {
    throw Fallback{"bad number"};
  }
  bool is_float = false;
  if (p < e && *p == '.') {
    ++p;
    if (p >= e || *p < '0' || *p > '9') throw Fallback{"bad fraction"};
    while (p < e && *p >= '0' && *p <= '9') ++p;
    is_float = true;
  }
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    if (p < e && (*p == '+' || *p == '-')) ++p;
    if (p >= e || *p < '0' || *p > '9') throw Fallback{"bad exponent"};
    while (p < e && *p >= '0' && *p <= '9') ++p;
    is_float = true;
  }
  c.p = p;
  const size_t n = static_cast<size_t>(p - b);
  if (!is_float) {
    PyObject* v = parse_int_text(b, n, scratch);  // int(text): arbitrary size, CPython's digit limit
    if (!v) throw Fallback{"int() rejected"};
    return v;
  }
  scratch.assign(b, n);
  double d = PyOS_string_to_double(scratch.c_str(), nullptr, nullptr);  // float(text): overflow -> inf
  if (d == -1.0 && PyErr_Occurred()) {
    PyErr_Clear();
    throw Fallback{"float() rejected"};
  }
  return PyFloat_FromDouble(d);
}

PyObject* loads_value(Cursor& c, std::string& scratch, int depth) {
  const char ch = c.peek();
  if (ch == '"') return loads_string(c, scratch);
  if (ch == '{') {
    if (depth >= kMaxDepth) throw Fallback{"too deep"};
    ++c.p;
    Ref d{PyDict_New()};
    if (!d.o) throw Fallback{"out of memory"};
    if (c.consume('}')) return d.release();
    for (;;) {
      if (c.peek() != '"') throw Fallback{"expected key"};
      Ref k{loads_string(c, scratch)};
      c.expect(':');
      Ref v{loads_value(c, scratch, depth + 1)};
      if (PyDict_SetItem(d.o, k.o, v.o) < 0) {
        PyErr_Clear();
        throw Fallback{"dict insert failed"};
      }
      if (c.consume(',')) continue;
      c.expect('}');
      return d.release();
    }
  }
  if (ch == '[') {
    if (depth >= kMaxDepth) throw Fallback{"too deep"};
    ++c.p;
    Ref l{PyList_New(0)};
    if (!l.o) throw Fallback{"out of memory"};
    if (c.consume(']')) return l.release();
    for (;;) {
      Ref v{loads_value(c, scratch, depth + 1)};
      if (PyList_Append(l.o, v.o) < 0) {
        PyErr_Clear();
        throw Fallback{"list append failed"};
      }
      if (c.consume(',')) continue;
      c.expect(']');
      return l.release();
    }
  }
  const size_t left = static_cast<size_t>(c.end - c.p);
  auto lit = [&](const char* w, size_t n) { return left >= n && memcmp(c.p, w, n) == 0; };
  if (lit("true", 4)) {
    c.p += 4;
    Py_RETURN_TRUE;
  }
  if (lit("false", 5)) {
    c.p += 5;
    Py_RETURN_FALSE;
  }
  if (lit("null", 4)) {
    c.p += 4;
    Py_RETURN_NONE;
  }
  if (lit("NaN", 3)) {
    c.p += 3;
    return PyFloat_FromDouble(std::nan(""));
  }
  if (lit("Infinity", 8)) {
    c.p += 8;
    return PyFloat_FromDouble(HUGE_VAL);
  }
  return loads_number(c, scratch);
}

PyObject* loads(PyObject*, PyObject* obj) {
  const char* b = nullptr;
  Py_ssize_t n = 0;
  Py_buffer view;
  bool have_view = false;
  if (PyUnicode_Check(obj)) {
    b = PyUnicode_AsUTF8AndSize(obj, &n);  // fails on lone surrogates: json.loads handles those
    if (!b) {
      PyErr_Clear();
      PyErr_SetString(g_fallback, "str not representable as UTF-8");
      return nullptr;
    }
  } else if ((PyBytes_Check(obj) || PyByteArray_Check(obj)) && PyObject_GetBuffer(obj, &view, PyBUF_SIMPLE) == 0) {
    have_view = true;
    b = static_cast<const char*>(view.buf);
    n = view.len;
  } else {
    PyErr_Clear();
    PyErr_SetString(g_fallback, "not str, bytes or bytearray");  // json.loads' own TypeError
    return nullptr;
  }
  PyObject* out = nullptr;
  try {
    Cursor c{b, b + n};
    std::string scratch;
    Ref v{loads_value(c, scratch, 0)};
    c.ws();
    if (c.p != c.end) throw Fallback{"trailing data"};
    out = v.release();
  } catch (const Fallback& f) {
    if (PyErr_Occurred()) PyErr_Clear();
    PyErr_SetString(g_fallback, f.why);
  }
  if (have_view) PyBuffer_Release(&view);
  return out;
}

PyMethodDef methods[] = {
    {"scan_nodelist", scan_nodelist, METH_VARARGS, "Scan one NodeList page into a ScanResult."},
    {"prescan_nodelist", prescan_nodelist, METH_VARARGS, "Pass 1 of a NodeList page (GIL released) -> capsule."},
    {"scan_prescanned", scan_prescanned, METH_VARARGS, "Pass 2 of a prescanned page into a ScanResult."},
    {"dumps_indent2", dumps_indent2, METH_O, "json.dumps(obj, ensure_ascii=False, indent=2), natively."},
    {"loads", loads, METH_O, "json.loads(data) for documents it provably reads alike; else FallbackError."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_fastpath", "Native CPU hot path (NodeList scan, JSON emit).", -1,
                      methods};

}  // namespace

PyMODINIT_FUNC PyInit__fastpath(void) {
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  g_fallback = PyErr_NewException("_fastpath.FallbackError", PyExc_ValueError, nullptr);
  Py_INCREF(g_fallback);
  PyModule_AddObject(m, "FallbackError", g_fallback);
  k_name = PyUnicode_InternFromString("name");
  k_ready = PyUnicode_InternFromString("ready");
  k_gpus = PyUnicode_InternFromString("gpus");
  k_breakdown = PyUnicode_InternFromString("gpu_breakdown");
  k_labels = PyUnicode_InternFromString("labels");
  k_taints = PyUnicode_InternFromString("taints");
  k_key = PyUnicode_InternFromString("key");
  k_value = PyUnicode_InternFromString("value");
  k_effect = PyUnicode_InternFromString("effect");
  a_gpu_nodes = PyUnicode_InternFromString("gpu_nodes");
  a_ready_gpu_nodes = PyUnicode_InternFromString("ready_gpu_nodes");
  a_extras = PyUnicode_InternFromString("extras");
  a_items_seen = PyUnicode_InternFromString("items_seen");
  PyModule_AddStringConstant(m, "BUILD", "gfx950-host/x86_64");
  return m;
}
