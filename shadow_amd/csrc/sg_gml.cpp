// sg_gml.cpp -- GML ingest for the network graph (host C++).
//
// Mirrors the grammar of src/lib/gml-parser/src/parser.rs (nom) and the edge
// conversion of ShadowEdge::try_from (src/main/network/graph/mod.rs:72-111),
// the latency unit parser Time::<TimePrefix>::from_str + convert(Nano)
// (src/main/utility/units.rs:218-251, 377-438) and NetworkGraph::parse
// (graph/mod.rs:134-181).  Parser quirks kept on purpose:
//   * a value is tried as Int (digits only, i32) before Float
//     (parser.rs:212-230), so `packet_loss 0` is an Int and is rejected as
//     "not a float" (graph/mod.rs:95-98);
//   * floats are correctly rounded to f32 (Rust str::parse::<f32> == strtof);
//   * a repeated node id silently re-maps the id to the later node
//     (graph/mod.rs:157-162).
// Difference: a latency whose ns value overflows u64 is reported here as a
// parse error; the reference panics later in PathProperties::from
// (graph/mod.rs:336 `.unwrap()`).
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/shadow_gpu.h"

struct sg_gml {
  bool directed = false;
  std::vector<uint32_t> node_id;  // GML id per node index
  std::vector<uint32_t> esrc, edst;
  std::vector<uint64_t> elat;
  std::vector<float> eloss;
  std::unordered_map<uint32_t, uint32_t> id_to_index;
};

namespace {

struct ParseError {
  std::string msg;
};

enum class VT { Int, Float, Str };
struct Value {
  VT t;
  int32_t i = 0;
  float f = 0;
  std::string s;
};

struct Parser {
  const char* p;
  const char* end;

  bool at_end() const { return p >= end; }
  static bool is_space(char c) { return c == ' ' || c == '\t'; }
  static bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
  [[noreturn]] void fail(const std::string& m) {
    throw ParseError{m + " at byte " + std::to_string((size_t)(p - start))};
  }
  const char* start;

  void space0() {
    while (!at_end() && is_space(*p)) p++;
  }
  void multispace0() {
    while (!at_end() && is_ws(*p)) p++;
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
    space0();
    return true;
  }
  bool tag(const char* t) {
    size_t n = strlen(t);
    if ((size_t)(end - p) >= n && memcmp(p, t, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  // key: [A-Za-z_][A-Za-z0-9_]* (parser.rs:42-49)
  bool key(std::string& out) {
    if (at_end() || !(isalpha((unsigned char)*p) || *p == '_')) return false;
    const char* s = p++;
    while (!at_end() && (isalnum((unsigned char)*p) || *p == '_')) p++;
    out.assign(s, p);
    return true;
  }
  // value (parser.rs:212-219): space0 then int|float|string, each followed by newline
  Value value() {
    space0();
    const char* s = p;
    // int: digit1 parsed as i32
    {
      const char* q = p;
      while (q < end && isdigit((unsigned char)*q)) q++;
      if (q > p) {
        std::string digits(p, q);
        errno = 0;
        char* e = nullptr;
        long long v = strtoll(digits.c_str(), &e, 10);
        bool ok = errno == 0 && v <= INT32_MAX;
        const char* save = p;
        p = q;
        if (ok && newline()) {
          Value r;
          r.t = VT::Int;
          r.i = (int32_t)v;
          return r;
        }
        p = save;
      }
    }
    // float: nom recognize_float: [+-]? (digits (. digits?)? | . digits) ([eE][+-]?digits)?
    {
      const char* q = p;
      if (q < end && (*q == '+' || *q == '-')) q++;
      const char* d0 = q;
      while (q < end && isdigit((unsigned char)*q)) q++;
      bool int_part = q > d0;
      bool frac = false;
      if (q < end && *q == '.') {
        const char* f0 = q + 1;
        const char* f = f0;
        while (f < end && isdigit((unsigned char)*f)) f++;
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
          while (x < end && isdigit((unsigned char)*x)) x++;
          if (x > x0) q = x;
        }
        std::string txt(p, q);
        const char* save = p;
        p = q;
        if (newline()) {
          Value r;
          r.t = VT::Float;
          r.f = strtof(txt.c_str(), nullptr);  // correctly rounded, as str::parse::<f32>
          return r;
        }
        p = save;
      }
    }
    // string: "..." with \\ and \" escapes (parser.rs:233-242)
    if (!at_end() && *p == '"') {
      p++;
      std::string out;
      while (!at_end() && *p != '"') {
        if (*p == '\\' && p + 1 < end && (p[1] == '\\' || p[1] == '"')) {
          out.push_back(p[1]);
          p += 2;
        } else {
          out.push_back(*p++);
        }
      }
      if (at_end()) fail("unterminated string");
      p++;
      if (!newline()) fail("expected newline after string");
      Value r;
      r.t = VT::Str;
      r.s = std::move(out);
      return r;
    }
    p = s;
    fail("expected a value");
  }
  // node/edge body: space0 "[" newline many_till((key, value), "]") newline
  std::unordered_map<std::string, Value> block() {
    space0();
    if (!tag("[")) fail("expected '['");
    if (!newline()) fail("expected newline after '['");
    std::unordered_map<std::string, Value> kv;
    size_t count = 0;
    for (;;) {
      if (tag("]")) break;
      std::string k;
      if (!key(k)) fail("expected key or ']'");
      Value v = value();
      count++;
      kv[k] = std::move(v);
    }
    if (kv.size() != count) fail("Duplicate keys are not supported");
    if (!newline()) fail("expected newline after ']'");
    return kv;
  }
};

// Time::<TimePrefix>::from_str (units.rs:411-438): returns (value, ns factor).
struct TimeVal {
  uint64_t value;
  uint64_t factor;
};

TimeVal parse_time(const std::string& s_in, const char* what) {
  // regex ^([+-]?[0-9\.]*)\s*(.*)$ ; both groups trimmed
  size_t i = 0;
  if (i < s_in.size() && (s_in[i] == '+' || s_in[i] == '-')) i++;
  while (i < s_in.size() && (isdigit((unsigned char)s_in[i]) || s_in[i] == '.')) i++;
  auto trim = [](std::string x) {
    size_t a = 0, b = x.size();
    while (a < b && isspace((unsigned char)x[a])) a++;
    while (b > a && isspace((unsigned char)x[b - 1])) b--;
    return x.substr(a, b - a);
  };
  std::string num = trim(s_in.substr(0, i)), unit = trim(s_in.substr(i));
  const std::string pre = std::string("Edge '") + what + "' is not a valid unit: ";
  // TimePrefix::from_str (units.rs:233-251); "" -> default Sec (:227-231)
  uint64_t factor;
  if (unit.empty())
    factor = 1000000000ull;
  else if (unit == "ns" || unit == "nanosecond" || unit == "nanoseconds")
    factor = 1;
  else if (unit == "us" || unit == "\xce\xbcs" || unit == "microsecond" || unit == "microseconds")
    factor = 1000;
  else if (unit == "ms" || unit == "millisecond" || unit == "milliseconds")
    factor = 1000000;
  else if (unit == "s" || unit == "sec" || unit == "secs" || unit == "second" || unit == "seconds")
    factor = 1000000000ull;
  else if (unit == "m" || unit == "min" || unit == "mins" || unit == "minute" || unit == "minutes")
    factor = 60000000000ull;
  else if (unit == "h" || unit == "hr" || unit == "hrs" || unit == "hour" || unit == "hours")
    factor = 3600000000000ull;
  else
    throw ParseError{pre + "Unit was not one of (ns|nanosecond|nanoseconds|us|\xce\xbcs|microsecond|"
                           "microseconds|ms|millisecond|milliseconds|s|sec|secs|second|seconds|m|min|"
                           "mins|minute|minutes|h|hr|hrs|hour|hours)"};
  // u64::from_str: optional '+', decimal digits only, no overflow
  std::string digits = num;
  if (!digits.empty() && digits[0] == '+') digits = digits.substr(1);
  if (digits.empty()) throw ParseError{pre + "cannot parse integer from empty string"};
  for (char c : digits)
    if (!isdigit((unsigned char)c)) throw ParseError{pre + "invalid digit found in string"};
  unsigned __int128 v = 0;
  for (char c : digits) {
    v = v * 10 + (unsigned)(c - '0');
    if (v > UINT64_MAX) throw ParseError{pre + "number too large to fit in target type"};
  }
  return TimeVal{(uint64_t)v, factor};
}

void parse_into(const char* text, size_t len, sg_gml* g) {
  Parser P{text, text + len, text};
  // gml (parser.rs:67-143)
  P.multispace0();
  if (!P.tag("graph")) P.fail("expected 'graph'");
  P.space0();
  if (!P.tag("[")) P.fail("expected '['");
  if (!P.newline()) P.fail("expected newline");
  std::vector<std::unordered_map<std::string, Value>> nodes, edges;
  std::unordered_map<std::string, int> others;
  int n_directed = 0;
  for (;;) {
    if (P.tag("]")) break;
    std::string k;
    if (!P.key(k)) P.fail("expected key or ']'");
    if (k == "node") {
      nodes.push_back(P.block());
      auto it = nodes.back().find("id");  // parser.rs:160-164
      if (it != nodes.back().end() && it->second.t != VT::Int) P.fail("Incorrect 'id' type");
    } else if (k == "edge") {
      edges.push_back(P.block());
      auto& kv = edges.back();  // parser.rs:190-202
      auto s = kv.find("source"), t = kv.find("target");
      if (s == kv.end()) P.fail("'source' doesn't exist");
      if (s->second.t != VT::Int) P.fail("Incorrect 'source' type");
      if (t == kv.end()) P.fail("'target' doesn't exist");
      if (t->second.t != VT::Int) P.fail("Incorrect 'target' type");
    } else if (k == "directed") {
      Value v = P.value();
      if (v.t != VT::Int) P.fail("Value was not an integer");
      if (v.i != 0 && v.i != 1) P.fail("Bool must be 0 or 1");
      g->directed = v.i == 1;
      n_directed++;
    } else {
      (void)P.value();
      if (others[k]++) P.fail("Duplicate keys are not supported");
    }
  }
  if (n_directed > 1) throw ParseError{"The 'directed' key must only be specified once"};
  // nodes (parser.rs:146-170; ShadowNode::try_from graph/mod.rs:28-60)
  for (auto& kv : nodes) {
    auto it = kv.find("id");
    if (it == kv.end()) throw ParseError{"Node 'id' was not provided"};
    for (const char* bw : {"host_bandwidth_down", "host_bandwidth_up"}) {
      auto b = kv.find(bw);
      if (b != kv.end() && b->second.t != VT::Str)
        throw ParseError{std::string("Node '") + bw + "' is not a string"};
    }
    uint32_t id = (uint32_t)it->second.i;
    uint32_t idx = (uint32_t)g->node_id.size();
    g->node_id.push_back(id);
    g->id_to_index[id] = idx;  // later duplicate wins (graph/mod.rs:157-162)
  }
  // edges: ShadowEdge::try_from order (graph/mod.rs:72-111), then endpoint lookup (:164-175)
  for (auto& kv : edges) {
    auto l = kv.find("latency");
    if (l == kv.end()) throw ParseError{"Edge 'latency' was not provided"};
    if (l->second.t != VT::Str) throw ParseError{"Edge 'latency' is not a string"};
    TimeVal lat = parse_time(l->second.s, "latency");
    auto j = kv.find("jitter");
    if (j != kv.end()) {
      if (j->second.t != VT::Str) throw ParseError{"Edge 'jitter' is not a string"};
      (void)parse_time(j->second.s, "jitter");  // parsed, then unused
    }
    float loss = 0.0f;
    auto pl = kv.find("packet_loss");
    if (pl != kv.end()) {
      if (pl->second.t != VT::Float) throw ParseError{"Edge 'packet_loss' is not a float"};
      loss = pl->second.f;
    }
    if (loss < 0.0f || loss > 1.0f) throw ParseError{"Edge 'packet_loss' is not in the range [0,1]"};
    if (lat.value == 0) throw ParseError{"Edge 'latency' must not be 0"};
    unsigned __int128 ns = (unsigned __int128)lat.value * lat.factor;
    if (ns > UINT64_MAX)  // reference: convert(Nano).unwrap() panics (graph/mod.rs:336)
      throw ParseError{"Edge 'latency': The resulting value is outside of the bounds [0, 18446744073709551615]"};
    uint32_t sid = (uint32_t)kv["source"].i, tid = (uint32_t)kv["target"].i;
    auto si = g->id_to_index.find(sid);
    if (si == g->id_to_index.end()) throw ParseError{"Edge source " + std::to_string(sid) + " doesn't exist"};
    auto ti = g->id_to_index.find(tid);
    if (ti == g->id_to_index.end()) throw ParseError{"Edge target " + std::to_string(tid) + " doesn't exist"};
    g->esrc.push_back(si->second);
    g->edst.push_back(ti->second);
    g->elat.push_back((uint64_t)ns);
    g->eloss.push_back(loss);
  }
}

}  // namespace

extern "C" {

int32_t sg_gml_parse(const char* text, size_t len, sg_gml** out, char* err, size_t err_len) {
  if (!out || (!text && len)) return SG_ERR_INVALID_ARG;
  *out = nullptr;
  sg_gml* g = new (std::nothrow) sg_gml();
  if (!g) return SG_ERR_OOM;
  try {
    parse_into(text ? text : "", len, g);
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
  }
  *out = g;
  return SG_OK;
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
  auto it = g->id_to_index.find(gml_id);
  if (it == g->id_to_index.end()) return SG_ERR_INVALID_ARG;
  *out_index = it->second;
  return SG_OK;
}

void sg_gml_destroy(sg_gml* g) { delete g; }

}  // extern "C"
