// sg_gml.cpp -- GML ingest for the network graph (host C++, multi-threaded).
//
// Mirrors the grammar of src/lib/gml-parser/src/parser.rs (nom) and the edge
// conversion of ShadowEdge::try_from (src/main/network/graph/mod.rs:72-111),
// the latency unit parser Time::<TimePrefix>::from_str + convert(Nano)
// (src/main/utility/units.rs:218-251, 377-438) and NetworkGraph::parse
// (graph/mod.rs:134-181).  Parser quirks kept on purpose:
//   * a value is tried as Int (digits only, i32) before Float
//     (parser.rs:212-230), so `packet_loss 0` is an Int and is rejected as
//     "not a float" (graph/mod.rs:95-98);
//   * floats are correctly rounded to f32 (Rust str::parse::<f32>, here
//     std::from_chars);
//   * a repeated node id silently re-maps the id to the later node
//     (graph/mod.rs:157-162).
// Difference: a latency whose ns value overflows u64 is reported here as a
// parse error; the reference panics later in PathProperties::from
// (graph/mod.rs:336 `.unwrap()`).
//
// Speed: no allocation per item -- keys and strings are
// spans into the text, a block's pairs live in a reused array -- and the
// body is split over threads.  Each thread starts at a guessed item boundary
// (a line whose key is `node` / `edge` followed by `[`) and parses whole items
// up to the next thread's start.  The boundaries are then verified in
// document order: a chunk that started at a true boundary and ended exactly on
// the next chunk's start proves that start true; a chunk that overshot (the
// next guess was inside a string) is continued on the calling thread until it
// lands on a later guess.  The result, including which error is reported
// first, is the single-threaded parse's.
#include <algorithm>
#include <dlfcn.h>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/shadow_gpu.h"

struct sg_gml {
  bool directed = false;
  std::vector<uint32_t> node_id;  // GML id per node index
  std::vector<uint32_t> esrc, edst;
  std::vector<uint64_t> elat;
  std::vector<float> eloss;
  // id -> index: a dense table when the ids are small, else a hash map
  std::vector<uint32_t> dense;
  std::unordered_map<uint32_t, uint32_t> sparse;
  bool lookup(uint32_t id, uint32_t& idx) const {
    if (!dense.empty()) {
      if (id >= dense.size() || dense[id] == UINT32_MAX) return false;
      idx = dense[id];
      return true;
    }
    auto it = sparse.find(id);
    if (it == sparse.end()) return false;
    idx = it->second;
    return true;
  }
};

namespace {

struct ParseError {
  std::string msg;
};

struct Span {
  const char* p = nullptr;
  uint32_t n = 0;
  bool eq(const char* s, uint32_t len) const { return n == len && memcmp(p, s, len) == 0; }
};

enum VT : uint8_t { V_INT, V_FLOAT, V_STR };
struct Value {
  VT t = V_INT;
  bool esc = false;  // the string holds \\ or \" escapes (s is the raw text between the quotes)
  int32_t i = 0;
  float f = 0;
  Span s;
};

std::string unescape(const Span& s, bool esc) {
  if (!esc) return std::string(s.p, s.n);
  std::string out;
  out.reserve(s.n);
  for (uint32_t k = 0; k < s.n; k++) {
    if (s.p[k] == '\\' && k + 1 < s.n && (s.p[k + 1] == '\\' || s.p[k + 1] == '"')) k++;
    out.push_back(s.p[k]);
  }
  return out;
}

inline bool is_space(char c) { return c == ' ' || c == '\t'; }
inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

// str::parse::<f32> of a recognize_float match [b, e): correctly rounded.
// Fast path (the usual "0.0123"): up to 19 significant digits and a decimal
// exponent within +-22 give the correctly rounded double m * 10^e exactly
// (both operands are exact doubles); its f32 rounding is the decimal's unless
// the double sits exactly on an f32 rounding midpoint, which goes to the slow
// path.  The slow path is std::from_chars (correctly rounded too), which in
// this libstdc++ serialises threads on the locale, hence the fast path.
bool parse_f32_slow(const char* b, const char* e, float& out) {
  std::string t;
  if (b < e && *b == '+') b++;  // from_chars takes no '+'
  const int neg = (b < e && *b == '-') ? 1 : 0;
  if (b + neg < e && b[neg] == '.') {  // ".5" / "-.5": from_chars wants a digit first
    t.assign(neg ? "-0" : "0");
    t.append(b + neg, e);
    b = t.data();
    e = t.data() + t.size();
  }
  auto r = std::from_chars(b, e, out, std::chars_format::general);
  if (r.ptr != e) return false;
  if (r.ec == std::errc::result_out_of_range) out = strtof(std::string(b, e).c_str(), nullptr);  // +-inf / 0
  return true;
}

bool parse_f32(const char* b, const char* e, float& out) {
  static const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  const char* q = b;
  bool neg = false;
  if (q < e && (*q == '+' || *q == '-')) neg = *q++ == '-';
  uint64_t m = 0;
  int nd = 0, e10 = 0;
  bool seen_dot = false;
  for (; q < e && (is_digit(*q) || *q == '.'); q++) {
    if (*q == '.') {
      seen_dot = true;
      continue;
    }
    if (m == 0 && *q == '0') {  // leading zeros are not significant
      if (seen_dot) e10--;
      continue;
    }
    if (nd == 19) return parse_f32_slow(b, e, out);
    m = m * 10 + (uint64_t)(*q - '0');
    nd++;
    if (seen_dot) e10--;
  }
  if (q < e) {  // [eE][+-]?digits (recognize_float guarantees the shape)
    q++;
    bool eneg = false;
    if (q < e && (*q == '+' || *q == '-')) eneg = *q++ == '-';
    int x = 0;
    for (; q < e; q++) {
      if (x > 100000) return parse_f32_slow(b, e, out);
      x = x * 10 + (*q - '0');
    }
    e10 += eneg ? -x : x;
  }
  if (m == 0) {
    out = neg ? -0.0f : 0.0f;
    return true;
  }
  if (m > (1ull << 53) || e10 < -22 || e10 > 22) return parse_f32_slow(b, e, out);
  double d = (double)m;
  d = e10 < 0 ? d / p10[-e10] : d * p10[e10];
  uint64_t u;
  memcpy(&u, &d, 8);
  const int bexp = (int)((u >> 52) & 0x7ff) - 1023;
  if (bexp < -125 || bexp > 126) return parse_f32_slow(b, e, out);  // f32 subnormal / overflow range
  if ((u & 0x1fffffffull) == 0x10000000ull) return parse_f32_slow(b, e, out);  // an f32 midpoint
  out = (float)(neg ? -d : d);
  return true;
}

struct KV {
  Span k;
  Value v;
};

struct Parser {
  const char* p;
  const char* end;
  const char* start;  // the whole text, for byte offsets in messages

  bool at_end() const { return p >= end; }
  [[noreturn]] void fail(const char* m) {
    throw ParseError{std::string(m) + " at byte " + std::to_string((size_t)(p - start))};
  }
  void space0() {
    while (p < end && is_space(*p)) p++;
  }
  void multispace0() {
    while (p < end && is_ws(*p)) p++;
  }
  // newline = space0 multispace1 space0 (parser.rs:243-245)
  bool newline() {
    const char* s = p;
    space0();
    const char* q = p;
    multispace0();
    if (p == q) {
      p = s;
      return false;
    }
    return true;
  }
  bool tag(char c) {
    if (p < end && *p == c) {
      p++;
      return true;
    }
    return false;
  }
  // key: [A-Za-z_][A-Za-z0-9_]* (parser.rs:42-49)
  bool key(Span& out) {
    if (at_end() || !(is_alpha(*p) || *p == '_')) return false;
    const char* s = p++;
    while (p < end && (is_alpha(*p) || is_digit(*p) || *p == '_')) p++;
    out.p = s;
    out.n = (uint32_t)(p - s);
    return true;
  }
  // value (parser.rs:212-219): space0 then int|float|string, each followed by newline
  Value value() {
    space0();
    Value r;
    {  // int: digit1 parsed as i32
      const char* q = p;
      while (q < end && is_digit(*q)) q++;
      if (q > p) {
        int64_t v = 0;
        bool ok = q - p <= 10;
        for (const char* d = p; ok && d < q; d++) v = v * 10 + (*d - '0');
        ok = ok && v <= INT32_MAX;
        const char* save = p;
        p = q;
        if (ok && newline()) {
          r.t = V_INT;
          r.i = (int32_t)v;
          return r;
        }
        p = save;
      }
    }
    {  // float: nom recognize_float: [+-]? (digits (. digits?)? | . digits) ([eE][+-]?digits)?
      const char* q = p;
      if (q < end && (*q == '+' || *q == '-')) q++;
      const char* d0 = q;
      while (q < end && is_digit(*q)) q++;
      const bool int_part = q > d0;
      bool frac = false;
      if (q < end && *q == '.') {
        const char* f0 = q + 1;
        const char* f = f0;
        while (f < end && is_digit(*f)) f++;
        if (int_part || f > f0) {
          frac = f > f0;
          q = f;
        }
      }
      if (int_part || frac) {
        if (q < end && (*q == 'e' || *q == 'E')) {
          const char* x = q + 1;
          if (x < end && (*x == '+' || *x == '-')) x++;
          const char* x0 = x;
          while (x < end && is_digit(*x)) x++;
          if (x > x0) q = x;
        }
        const char* save = p;
        float f = 0;
        const bool ok = parse_f32(p, q, f);
        p = q;
        if (ok && newline()) {
          r.t = V_FLOAT;
          r.f = f;
          return r;
        }
        p = save;
      }
    }
    if (!at_end() && *p == '"') {  // string: "..." with \\ and \" escapes (parser.rs:233-242)
      const char* s = ++p;
      bool esc = false;
      while (p < end && *p != '"') {
        if (*p == '\\' && p + 1 < end && (p[1] == '\\' || p[1] == '"')) {
          esc = true;
          p += 2;
        } else {
          p++;
        }
      }
      if (at_end()) fail("unterminated string");
      r.s.p = s;
      r.s.n = (uint32_t)(p - s);
      p++;
      if (!newline()) fail("expected newline after string");
      r.t = V_STR;
      r.esc = esc;
      return r;
    }
    fail("expected a value");
  }
  // node/edge body: space0 "[" newline many_till((key, value), "]") newline
  void block(std::vector<KV>& kv) {
    space0();
    if (!tag('[')) fail("expected '['");
    if (!newline()) fail("expected newline after '['");
    kv.clear();
    for (;;) {
      if (tag(']')) break;
      KV e;
      if (!key(e.k)) fail("expected key or ']'");
      e.v = value();
      kv.push_back(e);
    }
    for (size_t a = 1; a < kv.size(); a++)
      for (size_t b = 0; b < a; b++)
        if (kv[a].k.n == kv[b].k.n && memcmp(kv[a].k.p, kv[b].k.p, kv[a].k.n) == 0)
          fail("Duplicate keys are not supported");
    if (!newline()) fail("expected newline after ']'");
  }
};

const KV* find(const std::vector<KV>& kv, const char* k) {
  const uint32_t n = (uint32_t)strlen(k);
  for (const KV& e : kv)
    if (e.k.eq(k, n)) return &e;
  return nullptr;
}

// Time::<TimePrefix>::from_str (units.rs:411-438): the value and its ns
// factor, or a message in err.
bool parse_time(const char* s, size_t len, const char* what, uint64_t& value, uint64_t& factor, std::string& err) {
  // regex ^([+-]?[0-9\.]*)\s*(.*)$ ; both groups trimmed
  size_t i = 0;
  if (i < len && (s[i] == '+' || s[i] == '-')) i++;
  while (i < len && (is_digit(s[i]) || s[i] == '.')) i++;
  auto trim = [](const char*& a, const char*& b) {
    while (a < b && isspace((unsigned char)*a)) a++;
    while (b > a && isspace((unsigned char)b[-1])) b--;
  };
  const char *n0 = s, *n1 = s + i, *u0 = s + i, *u1 = s + len;
  trim(n0, n1);
  trim(u0, u1);
  const size_t ul = (size_t)(u1 - u0);
  auto is = [&](const char* w) { return ul == strlen(w) && memcmp(u0, w, ul) == 0; };
  auto fail = [&](const char* m) {
    err = std::string("Edge '") + what + "' is not a valid unit: " + m;
    return false;
  };
  // TimePrefix::from_str (units.rs:233-251); "" -> default Sec (:227-231)
  if (ul == 0)
    factor = 1000000000ull;
  else if (is("ns") || is("nanosecond") || is("nanoseconds"))
    factor = 1;
  else if (is("us") || is("\xce\xbcs") || is("microsecond") || is("microseconds"))
    factor = 1000;
  else if (is("ms") || is("millisecond") || is("milliseconds"))
    factor = 1000000;
  else if (is("s") || is("sec") || is("secs") || is("second") || is("seconds"))
    factor = 1000000000ull;
  else if (is("m") || is("min") || is("mins") || is("minute") || is("minutes"))
    factor = 60000000000ull;
  else if (is("h") || is("hr") || is("hrs") || is("hour") || is("hours"))
    factor = 3600000000000ull;
  else
    return fail("Unit was not one of (ns|nanosecond|nanoseconds|us|\xce\xbcs|microsecond|"
                "microseconds|ms|millisecond|milliseconds|s|sec|secs|second|seconds|m|min|"
                "mins|minute|minutes|h|hr|hrs|hour|hours)");
  // u64::from_str: optional '+', decimal digits only, no overflow
  if (n0 < n1 && *n0 == '+') n0++;
  if (n0 == n1) return fail("cannot parse integer from empty string");
  for (const char* d = n0; d < n1; d++)
    if (!is_digit(*d)) return fail("invalid digit found in string");
  unsigned __int128 v = 0;
  for (const char* d = n0; d < n1; d++) {
    v = v * 10 + (unsigned)(*d - '0');
    if (v > UINT64_MAX) return fail("number too large to fit in target type");
  }
  value = (uint64_t)v;
  return true;
}

// A string value's text: the span itself, or its unescaped copy in `buf`.
inline std::pair<const char*, size_t> text_of(const Value& v, std::string& buf) {
  if (!v.esc) return {v.s.p, v.s.n};
  buf = unescape(v.s, true);
  return {buf.data(), buf.size()};
}

// ShadowEdge::try_from (graph/mod.rs:72-111): latency (ns) and loss, or a message.
bool edge_convert(const std::vector<KV>& kv, uint64_t& lat_ns, float& loss, std::string& err) {
  const KV* l = find(kv, "latency");
  if (!l) return err = "Edge 'latency' was not provided", false;
  if (l->v.t != V_STR) return err = "Edge 'latency' is not a string", false;
  uint64_t lv, lf;
  std::string buf;
  auto lt = text_of(l->v, buf);
  if (!parse_time(lt.first, lt.second, "latency", lv, lf, err)) return false;
  if (const KV* j = find(kv, "jitter")) {
    if (j->v.t != V_STR) return err = "Edge 'jitter' is not a string", false;
    uint64_t jv, jf;
    auto jt = text_of(j->v, buf);
    if (!parse_time(jt.first, jt.second, "jitter", jv, jf, err)) return false;  // parsed, then unused
  }
  loss = 0.0f;
  if (const KV* pl = find(kv, "packet_loss")) {
    if (pl->v.t != V_FLOAT) return err = "Edge 'packet_loss' is not a float", false;
    loss = pl->v.f;
  }
  if (loss < 0.0f || loss > 1.0f) return err = "Edge 'packet_loss' is not in the range [0,1]", false;
  if (lv == 0) return err = "Edge 'latency' must not be 0", false;
  const unsigned __int128 ns = (unsigned __int128)lv * lf;
  if (ns > UINT64_MAX)  // reference: convert(Nano).unwrap() panics (graph/mod.rs:336)
    return err = "Edge 'latency': The resulting value is outside of the bounds [0, 18446744073709551615]", false;
  lat_ns = (uint64_t)ns;
  return true;
}

// One run of top-level items, in document order.
struct Chunk {
  enum Stop { LIMIT, END, ERROR };
  Stop stop = LIMIT;
  const char* endp = nullptr;     // where parsing stopped (LIMIT: at or past the limit)
  std::string err;                // ERROR: the syntax-phase message
  std::vector<int64_t> node_id;   // -1: no id
  std::vector<uint8_t> node_bad;  // 1: host_bandwidth_down not a string, 2: ..._up
  std::vector<uint32_t> esrc_id, edst_id;
  std::vector<uint64_t> elat;
  std::vector<float> eloss;
  int64_t conv_err = -1;  // the first edge (chunk-local) whose conversion failed
  std::string conv_msg;
  std::vector<std::string> others;  // top-level keys other than node / edge / directed
  int n_directed = 0;
  bool directed = false;
};

// Parse top-level items from P.p until the limit (an item starting at or past
// it is left alone), the graph's closing "]", or an error.
void parse_items(Parser P, const char* limit, Chunk& c) {
  std::vector<KV> kv;
  kv.reserve(16);
  try {
    for (;;) {
      if (P.p >= limit) {
        c.stop = Chunk::LIMIT;
        break;
      }
      if (P.tag(']')) {
        c.stop = Chunk::END;
        break;
      }
      Span k;
      if (!P.key(k)) P.fail("expected key or ']'");
      if (k.eq("node", 4)) {
        P.block(kv);
        const KV* id = find(kv, "id");  // parser.rs:160-164
        if (id && id->v.t != V_INT) P.fail("Incorrect 'id' type");
        c.node_id.push_back(id ? (int64_t)(uint32_t)id->v.i : -1);
        uint8_t bad = 0;  // ShadowNode::try_from (graph/mod.rs:28-60)
        const KV* bd = find(kv, "host_bandwidth_down");
        const KV* bu = find(kv, "host_bandwidth_up");
        if (bd && bd->v.t != V_STR)
          bad = 1;
        else if (bu && bu->v.t != V_STR)
          bad = 2;
        c.node_bad.push_back(bad);
      } else if (k.eq("edge", 4)) {
        P.block(kv);
        const KV* s = find(kv, "source");  // parser.rs:190-202
        const KV* t = find(kv, "target");
        if (!s) P.fail("'source' doesn't exist");
        if (s->v.t != V_INT) P.fail("Incorrect 'source' type");
        if (!t) P.fail("'target' doesn't exist");
        if (t->v.t != V_INT) P.fail("Incorrect 'target' type");
        c.esrc_id.push_back((uint32_t)s->v.i);
        c.edst_id.push_back((uint32_t)t->v.i);
        uint64_t lat = 0;
        float loss = 0;
        if (c.conv_err < 0 && !edge_convert(kv, lat, loss, c.conv_msg)) c.conv_err = (int64_t)c.elat.size();
        c.elat.push_back(lat);
        c.eloss.push_back(loss);
      } else if (k.eq("directed", 8)) {
        const Value v = P.value();
        if (v.t != V_INT) P.fail("Value was not an integer");
        if (v.i != 0 && v.i != 1) P.fail("Bool must be 0 or 1");
        c.directed = v.i == 1;
        c.n_directed++;
      } else {
        (void)P.value();
        c.others.emplace_back(k.p, k.n);
      }
    }
  } catch (const ParseError& e) {
    c.stop = Chunk::ERROR;
    c.err = e.msg;
  }
  c.endp = P.p;
}

// The next guessed item boundary after q: the first non-blank text of a line
// is `node` or `edge`, then blanks and '['.
const char* resync(const char* q, const char* end) {
  while (q < end) {
    const char* nl = (const char*)memchr(q, '\n', (size_t)(end - q));
    if (!nl) return end;
    const char* k = nl + 1;
    while (k < end && is_space(*k)) k++;
    if (end - k >= 5 && (memcmp(k, "node", 4) == 0 || memcmp(k, "edge", 4) == 0)) {
      const char* b = k + 4;
      while (b < end && is_space(*b)) b++;
      if (b < end && *b == '[') return k;
    }
    q = nl + 1;
  }
  return end;
}

unsigned default_threads() {
  if (const char* e = getenv("SG_GML_THREADS")) return (unsigned)std::max(1, atoi(e));
  const unsigned h = std::thread::hardware_concurrency();
  return std::max(1u, std::min(h ? h : 1u, 16u));  // a GPU's CPU share on the box
}

void parse_into(const char* text, size_t len, unsigned threads, sg_gml* g) {
  Parser P{text, text + len, text};
  // gml (parser.rs:67-143)
  P.multispace0();
  if ((size_t)(P.end - P.p) < 5 || memcmp(P.p, "graph", 5) != 0) P.fail("expected 'graph'");
  P.p += 5;
  P.space0();
  if (!P.tag('[')) P.fail("expected '['");
  if (!P.newline()) P.fail("expected newline");
  const char* body = P.p;
  const char* end = text + len;
  const size_t body_len = (size_t)(end - body);
  // chunk starts: s[0] = body (a true boundary), then guesses; 1 MiB or more each
  size_t T = body_len < ((size_t)4 << 20) ? 1 : std::min<size_t>(threads, body_len >> 20);
  T = std::max<size_t>(T, 1);
  std::vector<const char*> s(T + 1);
  s[0] = body;
  for (size_t i = 1; i < T; i++) s[i] = std::max(s[i - 1], resync(body + body_len * i / T, end));
  s[T] = end + 1;  // past the text: the last chunk runs to the graph's "]"
  std::vector<Chunk> ch(T);
  auto run = [&](size_t i) { parse_items(Parser{s[i], end, text}, s[i + 1], ch[i]); };
  if (T == 1) {
    run(0);
  } else {
    std::vector<std::thread> pool;
    for (size_t i = 1; i < T; i++) pool.emplace_back(run, i);
    run(0);
    for (auto& t : pool) t.join();
  }
  // verify the chain in document order; an overshooting chunk goes on here
  std::vector<Chunk> seq;
  seq.reserve(T + 4);
  for (size_t i = 0;;) {
    seq.push_back(std::move(ch[i]));
    while (seq.back().stop == Chunk::LIMIT && seq.back().endp != s[i + 1]) {
      // overshot s[i + 1] (a guess inside a string): continue to the first later guess
      size_t j = i + 1;
      while (j < T && s[j] < seq.back().endp) j++;
      Chunk more;
      parse_items(Parser{seq.back().endp, end, text}, s[j], more);
      seq.push_back(std::move(more));
      i = j - 1;
    }
    if (seq.back().stop != Chunk::LIMIT) break;
    if (++i >= T) break;  // landed exactly on s[i]: chunk i parsed from a true boundary
  }
  // the syntax phase fails on the first error in document order
  for (auto& c : seq)
    if (c.stop == Chunk::ERROR) throw ParseError{c.err};
  int n_directed = 0;
  std::vector<const std::string*> others;
  for (auto& c : seq) {
    n_directed += c.n_directed;
    if (c.n_directed) g->directed = c.directed;
    for (auto& o : c.others) others.push_back(&o);
  }
  if (n_directed > 1) throw ParseError{"The 'directed' key must only be specified once"};
  std::sort(others.begin(), others.end(), [](const std::string* a, const std::string* b) { return *a < *b; });
  for (size_t k = 1; k < others.size(); k++)
    if (*others[k] == *others[k - 1]) throw ParseError{"Duplicate keys are not supported"};
  // nodes (ShadowNode::try_from, graph/mod.rs:28-60), in order
  size_t n_nodes = 0, n_edges = 0;
  for (auto& c : seq) {
    for (size_t k = 0; k < c.node_id.size(); k++) {
      if (c.node_id[k] < 0) throw ParseError{"Node 'id' was not provided"};
      if (c.node_bad[k] == 1) throw ParseError{"Node 'host_bandwidth_down' is not a string"};
      if (c.node_bad[k] == 2) throw ParseError{"Node 'host_bandwidth_up' is not a string"};
    }
    n_nodes += c.node_id.size();
    n_edges += c.elat.size();
  }
  g->node_id.resize(n_nodes);
  uint32_t max_id = 0;
  {
    size_t o = 0;
    for (auto& c : seq)
      for (int64_t id : c.node_id) {
        g->node_id[o++] = (uint32_t)id;
        max_id = std::max(max_id, (uint32_t)id);
      }
  }
  // id -> index, a later duplicate winning (graph/mod.rs:157-162)
  if (n_nodes && (uint64_t)max_id < 4 * (uint64_t)n_nodes + 1024) {
    g->dense.assign((size_t)max_id + 1, UINT32_MAX);
    for (uint32_t k = 0; k < n_nodes; k++) g->dense[g->node_id[k]] = k;
  } else {
    g->sparse.reserve(n_nodes);
    for (uint32_t k = 0; k < n_nodes; k++) g->sparse[g->node_id[k]] = k;
  }
  // edges: conversion, then endpoint lookup (graph/mod.rs:164-175), in order;
  // chunks run on threads, the first failure in document order wins
  g->esrc.resize(n_edges);
  g->edst.resize(n_edges);
  g->elat.resize(n_edges);
  g->eloss.resize(n_edges);
  std::vector<size_t> eoff(seq.size() + 1, 0);
  for (size_t k = 0; k < seq.size(); k++) eoff[k + 1] = eoff[k] + seq[k].elat.size();
  std::vector<std::string> first_err(seq.size());
  auto link = [&](size_t k) {
    const Chunk& c = seq[k];
    const size_t o = eoff[k], n = c.elat.size();
    for (size_t e = 0; e < n; e++) {
      if ((int64_t)e == c.conv_err) {
        first_err[k] = c.conv_msg;
        return;
      }
      uint32_t si, ti;
      if (!g->lookup(c.esrc_id[e], si)) {
        first_err[k] = "Edge source " + std::to_string(c.esrc_id[e]) + " doesn't exist";
        return;
      }
      if (!g->lookup(c.edst_id[e], ti)) {
        first_err[k] = "Edge target " + std::to_string(c.edst_id[e]) + " doesn't exist";
        return;
      }
      g->esrc[o + e] = si;
      g->edst[o + e] = ti;
      g->elat[o + e] = c.elat[e];
      g->eloss[o + e] = c.eloss[e];
    }
  };
  if (seq.size() == 1) {
    link(0);
  } else {
    std::vector<std::thread> pool;
    for (size_t k = 1; k < seq.size(); k++) pool.emplace_back(link, k);
    link(0);
    for (auto& t : pool) t.join();
  }
  for (auto& m : first_err)
    if (!m.empty()) throw ParseError{m};
}

// ---- load_network_graph (graph/mod.rs:483-513): the file, plain or xz ------
//
// xz goes through the system liblzma (liblzma.so.5, the library Python's lzma
// module wraps; lzma_rs::xz_decompress in the reference), opened with dlopen: the
// image ships the library but not lzma.h, so the few entry points used are
// declared here from liblzma's public, stable ABI (lzma/base.h, lzma/container.h).
struct LzmaStream {  // lzma_stream
  const uint8_t* next_in;
  size_t avail_in;
  uint64_t total_in;
  uint8_t* next_out;
  size_t avail_out;
  uint64_t total_out;
  const void* allocator;
  void* internal;
  void* reserved_ptr[4];
  uint64_t reserved_int[2];
  size_t reserved_sz[2];
  int reserved_enum[2];
};
struct Lzma {
  int (*stream_decoder)(LzmaStream*, uint64_t memlimit, uint32_t flags);
  int (*code)(LzmaStream*, int action);
  void (*end)(LzmaStream*);
  bool ok = false;
  Lzma() {
    void* h = dlopen("liblzma.so.5", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    stream_decoder = (int (*)(LzmaStream*, uint64_t, uint32_t))dlsym(h, "lzma_stream_decoder");
    code = (int (*)(LzmaStream*, int))dlsym(h, "lzma_code");
    end = (void (*)(LzmaStream*))dlsym(h, "lzma_end");
    ok = stream_decoder && code && end;
  }
};
constexpr int LZMA_OK_ = 0, LZMA_STREAM_END_ = 1, LZMA_FINISH_ = 3;

// read_xz (graph/mod.rs:484-496): one .xz stream, decompressed whole
static std::string xz_decompress(const std::string& packed, const char* path) {
  static Lzma lz;
  if (!lz.ok) throw ParseError{std::string("Failed to decompress file: liblzma.so.5 not available (") + path + ")"};
  LzmaStream st;
  memset(&st, 0, sizeof(st));  // LZMA_STREAM_INIT
  if (lz.stream_decoder(&st, UINT64_MAX, 0) != LZMA_OK_) throw ParseError{"Failed to decompress file: decoder init"};
  std::string out;
  out.resize(std::max<size_t>(packed.size() * 4, 1 << 16));
  st.next_in = (const uint8_t*)packed.data();
  st.avail_in = packed.size();
  size_t done = 0;
  for (;;) {
    st.next_out = (uint8_t*)&out[done];
    st.avail_out = out.size() - done;
    const int rc = lz.code(&st, LZMA_FINISH_);
    done = out.size() - st.avail_out;
    if (rc == LZMA_STREAM_END_) break;
    if (rc != LZMA_OK_) {
      lz.end(&st);
      throw ParseError{"Failed to decompress file: liblzma error " + std::to_string(rc)};
    }
    if (!st.avail_out) out.resize(out.size() * 2);
    else if (!st.avail_in) {  // input ended inside the stream
      lz.end(&st);
      throw ParseError{"Failed to decompress file: truncated xz stream"};
    }
  }
  lz.end(&st);
  out.resize(done);
  return out;
}

// String::from_utf8 / read_to_string: well-formed UTF-8 (no overlong forms, no
// surrogates, nothing past U+10FFFF)
static bool utf8_valid(const std::string& t) {
  const unsigned char* p = (const unsigned char*)t.data();
  const size_t n = t.size();
  size_t i = 0;
  while (i < n) {
    while (i + 8 <= n) {  // ASCII fast path, 8 bytes at a time
      uint64_t w;
      memcpy(&w, p + i, 8);
      if (w & 0x8080808080808080ull) break;
      i += 8;
    }
    if (i >= n) break;
    const unsigned c = p[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    int len;
    unsigned lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) len = 2;
    else if (c >= 0xE0 && c <= 0xEF) {
      len = 3;
      if (c == 0xE0) lo = 0xA0;
      if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      len = 4;
      if (c == 0xF0) lo = 0x90;
      if (c == 0xF4) hi = 0x8F;
    } else {
      return false;
    }
    if (i + len > n) return false;
    if (p[i + 1] < lo || p[i + 1] > hi) return false;
    for (int k = 2; k < len; k++)
      if ((p[i + k] & 0xC0) != 0x80) return false;
    i += len;
  }
  return true;
}

static std::string read_file(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) throw ParseError{std::string("Failed to read file: ") + path};
  std::string t;
  char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) t.append(buf, k);
  const bool bad = ferror(f);
  fclose(f);
  if (bad) throw ParseError{std::string("Failed to read file: ") + path};
  return t;
}

}  // namespace

extern "C" {

int32_t sg_gml_load(const char* path, uint32_t compression, uint32_t threads, sg_gml** out, char* err,
                    size_t err_len) {
  if (!out || !path || compression > 1) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  std::string text;
  try {
    std::string p = path;
    if (p.size() >= 2 && p[0] == '~' && p[1] == '/' && getenv("HOME")) p = getenv("HOME") + p.substr(1);  // tilde_expansion
    text = read_file(p.c_str());
    if (compression == 1) text = xz_decompress(text, p.c_str());
    if (!utf8_valid(text))
      throw ParseError{compression == 1 ? "invalid utf-8 sequence (String::from_utf8)"
                                        : "Failed to read file: " + p + ": stream did not contain valid UTF-8"};
  } catch (const ParseError& e) {
    if (err && err_len) {
      strncpy(err, e.msg.c_str(), err_len - 1);
      err[err_len - 1] = 0;
    }
    return SG_ERR_PARSE;
  } catch (const std::bad_alloc&) {
    return SG_ERR_OOM;
  }
  return sg_gml_parse_threads(text.data(), text.size(), threads, out, err, err_len);
}

int32_t sg_gml_parse_threads(const char* text, size_t len, uint32_t threads, sg_gml** out, char* err,
                             size_t err_len) {
  if (!out || (!text && len)) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_gml* g = new (std::nothrow) sg_gml();
  if (!g) return SG_ERR_OOM;
  try {
    parse_into(text ? text : "", len, threads ? threads : default_threads(), g);
  } catch (const ParseError& e) {
    if (err && err_len) {
      strncpy(err, e.msg.c_str(), err_len - 1);
      err[err_len - 1] = 0;
    }
    delete g;
    return SG_ERR_PARSE;
  } catch (const std::bad_alloc&) {
    delete g;
    return SG_ERR_OOM;
  } catch (const std::system_error&) {  // no thread could be started
    delete g;
    return SG_ERR_OOM;
  }
  *out = g;
  return SG_OK;
}

int32_t sg_gml_parse(const char* text, size_t len, sg_gml** out, char* err, size_t err_len) {
  return sg_gml_parse_threads(text, len, 0, out, err, err_len);
}

int32_t sg_gml_graph(const sg_gml* g, sg_graph* out) {
  if (!g || !out) return SG_ERR_INVALID_ARG;
  out->n_nodes = (uint32_t)g->node_id.size();
  out->n_edges = (uint32_t)g->esrc.size();
  out->edge_src = g->esrc.data();
  out->edge_dst = g->edst.data();
  out->edge_latency_ns = g->elat.data();
  out->edge_packet_loss = g->eloss.data();
  out->node_gml_id = g->node_id.data();
  out->directed = g->directed ? 1 : 0;
  return SG_OK;
}

int32_t sg_gml_node_index(const sg_gml* g, uint32_t gml_id, uint32_t* out_index) {
  if (!g || !out_index) return SG_ERR_INVALID_ARG;
  return g->lookup(gml_id, *out_index) ? SG_OK : SG_ERR_INVALID_ARG;
}

void sg_gml_destroy(sg_gml* g) { delete g; }

}  // extern "C"
