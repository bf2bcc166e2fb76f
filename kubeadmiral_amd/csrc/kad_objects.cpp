// Native SchedulingUnit builder (include/kad_objects.h): federated objects and
// their propagation policies as JSON text → kad_su_columns.
//
// Per object, on the library's worker threads:
//   1. parse the JSON text into a flat node array (objects keep every member in order, duplicates
//      included: Go's decoder sees them all; the unstructured map view keeps the last);
//   2. MatchedPolicyKey (scheduler/util.go:37-49) → the policy, decoded once per batch;
//   3. schedulingUnitForFedObject (schedulingunit.go:38-163): the template's metadata, the scheduling
//      mode and DesiredReplicas, the current clusters (spec.placements + the global scheduler's replica
//      overrides, :181-222 and util/overrides.go:68-112), then every policy field with its annotation
//      override (:224-668).
// Then, serially in object order, the strings are interned into one table and the columns laid out.
//
// Decoding restates the Go 1.19 encoding/json rules kubeadmiral_amd/gojson.py restates (struct fields
// exact-then-case-folded, null, integer ranges, interface{} numbers as float64, an error anywhere fails
// the call); typed decodes of the object itself visit its members in the sorted key order of the
// unstructured round trip (UnstructuredToInterface). Parity: tests/test_native_objects.py compares
// every field with kubeadmiral_amd/objects.py and the reference's schedulingunit table.
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <optional>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/kad_objects.h"
#include "kad_pool.h"

namespace {

using sv = std::string_view;

// ------------------------------------------------------------------ constants (scheduler/constants.go,
// common/constants.go)
constexpr sv PREFIXED_GLOBAL_SCHEDULER = "kubeadmiral.io/global-scheduler";
constexpr sv POLICY_LABEL = "kubeadmiral.io/propagation-policy-name";
constexpr sv CLUSTER_POLICY_LABEL = "kubeadmiral.io/cluster-propagation-policy-name";
constexpr sv SCHEDULING_MODE_ANN = "kubeadmiral.io/scheduling-mode";
constexpr sv STICKY_ANN = "kubeadmiral.io/sticky-cluster";
constexpr sv TOLERATIONS_ANN = "kubeadmiral.io/tolerations";
constexpr sv PLACEMENTS_ANN = "kubeadmiral.io/placements";
constexpr sv SELECTOR_ANN = "kubeadmiral.io/clusterSelector";
constexpr sv AFFINITY_ANN = "kubeadmiral.io/affinity";
constexpr sv MAX_CLUSTERS_ANN = "kubeadmiral.io/maxClusters";
constexpr sv AUTO_MIGRATION_INFO_ANN = "kubeadmiral.io/auto-migration-info";
constexpr sv DUPLICATE = "Duplicate", DIVIDE = "Divide";
constexpr sv ENABLE_FOLLOWER_ANN = "internal.kubeadmiral.io/enable-follower-scheduling";
constexpr sv TRIGGER_HASH_ANN = "kubeadmiral.io/scheduling-trigger-hash";
constexpr sv NO_SCHEDULING_ANN = "kubeadmiral.io/no-scheduling";
constexpr sv FOLLOWS_OBJECT_ANN = "kubeadmiral.io/follows-object";
constexpr sv POD_UNSCHEDULABLE_THRESHOLD_ANN = "internal.kubeadmiral.io/pod-unschedulable-threshold";

struct Fail {  // the reference returns an error (status) or panics
  int status;
  std::string msg;
};
[[noreturn]] void fail(int st, std::string m) { throw Fail{st, std::move(m)}; }

// ------------------------------------------------------------------ JSON text → nodes
enum JT : uint8_t { J_NULL, J_FALSE, J_TRUE, J_NUM, J_STR, J_ARR, J_OBJ };
struct JV {
  JT t = J_NULL;
  bool isint = false;  // number: an integer literal (no fraction or exponent)
  bool fits = false;   //   ... within int64
  int64_t i = 0;
  double d = 0;        // number: the literal as float64 (±inf beyond range)
  uint32_t a = 0, n = 0;  // string: bytes s[a, a+n); array: kids[a, a+n); object: kids[a, a+2n) as (key, value)
};
struct JDoc {
  std::vector<JV> v;
  std::vector<uint32_t> kids;
  std::string s;
  sv str(uint32_t x) const { return sv(s.data() + v[x].a, v[x].n); }
};

struct Parser {
  const char* p;
  const char* e;
  JDoc& d;
  std::vector<uint32_t> stack;  // children of the open containers
  static constexpr int MAX_DEPTH = 1000;

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static void put_utf8(std::string& o, uint32_t c) {
    if (c < 0x80) {
      o += (char)c;
    } else if (c < 0x800) {
      o += (char)(0xC0 | (c >> 6));
      o += (char)(0x80 | (c & 0x3F));
    } else if (c < 0x10000) {
      o += (char)(0xE0 | (c >> 12));
      o += (char)(0x80 | ((c >> 6) & 0x3F));
      o += (char)(0x80 | (c & 0x3F));
    } else {
      o += (char)(0xF0 | (c >> 18));
      o += (char)(0x80 | ((c >> 12) & 0x3F));
      o += (char)(0x80 | ((c >> 6) & 0x3F));
      o += (char)(0x80 | (c & 0x3F));
    }
  }
  bool hex4(uint32_t* out) {
    if (e - p < 4) return false;
    uint32_t x = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = p[k];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    p += 4;
    *out = x;
    return true;
  }
  // a string (p at the opening quote) appended to d.s; unpaired surrogate escapes become U+FFFD
  // (Go's decoder; gojson._fix_str), control characters are an error (both decoders)
  bool str(uint32_t* a, uint32_t* n) {
    ++p;
    const size_t start = d.s.size();
    for (;;) {
      const char* q = p;
      while (q < e && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
      d.s.append(p, (size_t)(q - p));
      p = q;
      if (p >= e || (unsigned char)*p < 0x20) return false;
      if (*p == '"') {
        ++p;
        break;
      }
      ++p;  // backslash
      if (p >= e) return false;
      const char c = *p++;
      switch (c) {
        case '"': d.s += '"'; break;
        case '\\': d.s += '\\'; break;
        case '/': d.s += '/'; break;
        case 'b': d.s += '\b'; break;
        case 'f': d.s += '\f'; break;
        case 'n': d.s += '\n'; break;
        case 'r': d.s += '\r'; break;
        case 't': d.s += '\t'; break;
        case 'u': {
          uint32_t c1;
          if (!hex4(&c1)) return false;
          if (c1 >= 0xD800 && c1 < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t c2;
            if (hex4(&c2) && c2 >= 0xDC00 && c2 < 0xE000) {
              put_utf8(d.s, 0x10000 + ((c1 - 0xD800) << 10) + (c2 - 0xDC00));
              break;
            }
            p = save;  // not a low surrogate: c1 is unpaired, the next escape is read on its own
          }
          put_utf8(d.s, (c1 >= 0xD800 && c1 < 0xE000) ? 0xFFFDu : c1);
          break;
        }
        default: return false;
      }
    }
    *a = (uint32_t)start;
    *n = (uint32_t)(d.s.size() - start);
    return true;
  }
  bool num(JV& x) {
    const char* s0 = p;
    if (p < e && *p == '-') ++p;
    if (p >= e) return false;
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < e && *p >= '0' && *p <= '9') ++p;
    } else {
      return false;
    }
    bool isint = true;
    if (p < e && *p == '.') {
      ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
      isint = false;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
      isint = false;
    }
    std::string lit(s0, (size_t)(p - s0));
    x.t = J_NUM;
    x.isint = isint;
    x.d = std::strtod(lit.c_str(), nullptr);
    if (isint) {
      const bool neg = lit[0] == '-';
      const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
      uint64_t v = 0;
      bool ok = true;
      for (size_t k = neg ? 1 : 0; k < lit.size(); ++k) {
        const uint64_t dg = (uint64_t)(lit[k] - '0');
        if (v > (lim - dg) / 10) {
          ok = false;
          break;
        }
        v = v * 10 + dg;
      }
      x.fits = ok;
      x.i = ok ? (neg ? (int64_t)(0 - v) : (int64_t)v) : 0;
    }
    return true;
  }
  bool lit(const char* w, size_t n) {
    if ((size_t)(e - p) < n || std::memcmp(p, w, n) != 0) return false;
    p += n;
    return true;
  }
  // one value; its node index in *out
  bool value(uint32_t* out, int depth) {
    if (depth > MAX_DEPTH) return false;
    ws();
    if (p >= e) return false;
    JV x;
    const char c = *p;
    if (c == '{' || c == '[') {
      const bool obj = c == '{';
      ++p;
      const size_t base = stack.size();
      ws();
      const char close = obj ? '}' : ']';
      if (p < e && *p == close) {
        ++p;
      } else {
        for (;;) {
          if (obj) {
            ws();
            if (p >= e || *p != '"') return false;
            JV k;
            k.t = J_STR;
            if (!str(&k.a, &k.n)) return false;
            d.v.push_back(k);
            stack.push_back((uint32_t)(d.v.size() - 1));
            ws();
            if (p >= e || *p != ':') return false;
            ++p;
          }
          uint32_t ch;
          if (!value(&ch, depth + 1)) return false;
          stack.push_back(ch);
          ws();
          if (p < e && *p == ',') {
            ++p;
            continue;
          }
          if (p < e && *p == close) {
            ++p;
            break;
          }
          return false;
        }
      }
      x.t = obj ? J_OBJ : J_ARR;
      x.a = (uint32_t)d.kids.size();
      const size_t cnt = stack.size() - base;
      x.n = (uint32_t)(obj ? cnt / 2 : cnt);
      d.kids.insert(d.kids.end(), stack.begin() + (long)base, stack.end());
      stack.resize(base);
    } else if (c == '"') {
      x.t = J_STR;
      if (!str(&x.a, &x.n)) return false;
    } else if (c == 't') {
      if (!lit("true", 4)) return false;
      x.t = J_TRUE;
    } else if (c == 'f') {
      if (!lit("false", 5)) return false;
      x.t = J_FALSE;
    } else if (c == 'n') {
      if (!lit("null", 4)) return false;
      x.t = J_NULL;
    } else {
      if (!num(x)) return false;
    }
    d.v.push_back(x);
    *out = (uint32_t)(d.v.size() - 1);
    return true;
  }
};

// parse a whole text (one value, surrounding whitespace only); the root is d.v.back()
bool parse(sv text, JDoc& d, uint32_t* root) {
  d.v.clear();
  d.kids.clear();
  d.s.clear();
  Parser ps{text.data(), text.data() + text.size(), d, {}};
  if (!ps.value(root, 0)) return false;
  ps.ws();
  return ps.p == ps.e;
}

// ------------------------------------------------------------------ unstructured (map) view
// m[key] of a decoded map: the last member with that key (a Go / Python map keeps the last)
int64_t get(const JDoc& d, uint32_t obj, sv key) {
  if (d.v[obj].t != J_OBJ) return -1;
  const JV& o = d.v[obj];
  for (int64_t k = (int64_t)o.n - 1; k >= 0; --k)
    if (d.str(d.kids[o.a + 2 * k]) == key) return d.kids[o.a + 2 * k + 1];
  return -1;
}

// the members a typed decode visits: in text order (json.Unmarshal of text), or — for the object
// itself, re-read through UnstructuredToInterface — unique keys (last wins) sorted bytewise
void members(const JDoc& d, uint32_t obj, bool sorted_unique, std::vector<std::pair<sv, uint32_t>>& out) {
  out.clear();
  const JV& o = d.v[obj];
  for (uint32_t k = 0; k < o.n; ++k) out.emplace_back(d.str(d.kids[o.a + 2 * k]), d.kids[o.a + 2 * k + 1]);
  if (!sorted_unique || out.size() < 2) return;
  std::stable_sort(out.begin(), out.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  size_t w = 0;
  for (size_t r = 0; r < out.size(); ++r) {
    if (w > 0 && out[w - 1].first == out[r].first) out[w - 1] = out[r];  // later text position wins
    else out[w++] = out[r];
  }
  out.resize(w);
}

// bytes.EqualFold against an ASCII field name as gojson._fold does it: ASCII case, U+017F → s, U+212A → k
bool fold_eq(sv key, sv lower_field) {  // lower_field: compared lower-cased
  size_t i = 0, j = 0;
  while (i < key.size()) {
    const unsigned char c = (unsigned char)key[i];
    char f;
    if (c < 0x80) {
      f = (char)(c >= 'A' && c <= 'Z' ? c + 32 : c);
      i += 1;
    } else if (c == 0xC5 && i + 1 < key.size() && (unsigned char)key[i + 1] == 0xBF) {
      f = 's';
      i += 2;
    } else if (c == 0xE2 && i + 2 < key.size() && (unsigned char)key[i + 1] == 0x84 && (unsigned char)key[i + 2] == 0xAA) {
      f = 'k';
      i += 3;
    } else {
      return false;
    }
    const char g = lower_field[j < lower_field.size() ? j : 0];
    if (j >= lower_field.size() || (char)(g >= 'A' && g <= 'Z' ? g + 32 : g) != f) return false;
    ++j;
  }
  return j == lower_field.size();
}

// ------------------------------------------------------------------ Go typed decoding
struct Dec {
  const JDoc& d;
  bool sorted;  // member order: see members()
  // the first error (json.Unmarshal's result is discarded on any error, so decoding stops there): recorded,
  // not thrown — the annotation overrides that fail fall back silently and are common enough for C++
  // exceptions (serialised in the unwinder) to cost more than the decode
  const char* err = nullptr;

  void type_err(const char* want) {
    if (!err) err = want;
  }
  const JV& at(uint32_t x) const { return d.v[x]; }
  bool null(uint32_t x) const { return d.v[x].t == J_NULL; }

  // struct: visit each member matched to a field (exact name first, else case-folded; the first field of
  // that folded name); fields: their JSON names. null leaves the struct as it is
  template <size_t N, class F>
  void fields(uint32_t x, const sv (&names)[N], F&& on) {
    if (null(x) || err) return;
    if (at(x).t != J_OBJ) return type_err("struct");
    std::vector<std::pair<sv, uint32_t>> ms;
    members(d, x, sorted, ms);
    for (const auto& [key, val] : ms) {
      if (err) return;
      int f = -1;
      for (size_t k = 0; k < N && f < 0; ++k)
        if (names[k] == key) f = (int)k;
      for (size_t k = 0; k < N && f < 0; ++k)
        if (fold_eq(key, names[k])) f = (int)k;
      if (f >= 0) on(f, val);
    }
  }
  // null leaves string / bool / integer / struct values as they are
  void str(uint32_t x, std::string& out) {
    if (null(x)) return;
    if (at(x).t != J_STR) return type_err("string");
    out.assign(d.str(x));
  }
  void boolean(uint32_t x, bool& out) {
    if (null(x)) return;
    if (at(x).t != J_TRUE && at(x).t != J_FALSE) return type_err("bool");
    out = at(x).t == J_TRUE;
  }
  void int64(uint32_t x, int64_t& out) {
    if (null(x)) return;
    if (at(x).t != J_NUM || !at(x).isint || !at(x).fits) return type_err("int64");
    out = at(x).i;
  }
  void int32(uint32_t x, int32_t& out) {
    if (null(x)) return;
    const JV& v = at(x);
    if (v.t != J_NUM || !v.isint || !v.fits || v.i < INT32_MIN || v.i > INT32_MAX) return type_err("int32");
    out = (int32_t)v.i;
  }
  // *int64 / *string / *struct: null → nil, else decode into the pointee (a fresh zero when nil)
  void ptr_int64(uint32_t x, std::optional<int64_t>& out) {
    if (null(x)) {
      out.reset();
      return;
    }
    int64_t v = out.value_or(0);
    int64(x, v);
    out = v;
  }
  void ptr_str(uint32_t x, std::optional<std::string>& out) {
    if (null(x)) {
      out.reset();
      return;
    }
    std::string v = out.value_or(std::string());
    str(x, v);
    out = std::move(v);
  }
  // []T: null → nil, else a new slice of freshly decoded elements
  template <class T, class F>
  void slice(uint32_t x, std::optional<std::vector<T>>& out, F&& elem) {
    if (null(x)) {
      out.reset();
      return;
    }
    if (err) return;
    if (at(x).t != J_ARR) return type_err("slice");
    std::vector<T> v(at(x).n);
    for (uint32_t k = 0; k < at(x).n && !err; ++k) elem(d.kids[at(x).a + k], v[k]);
    out = std::move(v);
  }
  // map[string]T: null → nil, else the current map (or a new one) with every member set to a freshly
  // decoded value (insertion order kept; a repeated key keeps its first position)
  template <class T, class F>
  void map(uint32_t x, std::optional<std::vector<std::pair<std::string, T>>>& out, F&& elem) {
    if (null(x)) {
      out.reset();
      return;
    }
    if (err) return;
    if (at(x).t != J_OBJ) return type_err("map");
    std::vector<std::pair<std::string, T>> m = out ? std::move(*out) : std::vector<std::pair<std::string, T>>();
    std::unordered_map<std::string, size_t> pos;
    if (m.size() > 8)
      for (size_t k = 0; k < m.size(); ++k) pos.emplace(m[k].first, k);
    const JV& o = at(x);
    for (uint32_t k = 0; k < o.n && !err; ++k) {
      std::string key(d.str(d.kids[o.a + 2 * k]));
      T v{};
      elem(d.kids[o.a + 2 * k + 1], v);
      size_t at_ = SIZE_MAX;
      if (m.size() > 8 || !pos.empty()) {
        if (pos.empty())
          for (size_t q = 0; q < m.size(); ++q) pos.emplace(m[q].first, q);
        auto it = pos.find(key);
        if (it != pos.end()) at_ = it->second;
      } else {
        for (size_t q = 0; q < m.size(); ++q)
          if (m[q].first == key) at_ = q;
      }
      if (at_ != SIZE_MAX) {
        m[at_].second = std::move(v);
      } else {
        if (!pos.empty()) pos.emplace(key, m.size());
        m.emplace_back(std::move(key), std::move(v));
      }
    }
    out = std::move(m);
  }
  // interface{}: validated (numbers must be finite float64s); kind and float value kept
  struct Any {
    JT t = J_NULL;
    double f = 0;
  };
  void any(uint32_t x, Any& out) {
    const JV& v = at(x);
    out.t = v.t;
    if (v.t == J_NUM) {
      if (!std::isfinite(v.d) && !err) err = "number out of range";
      out.f = v.d;
    } else if (v.t == J_ARR) {
      Any sub;
      for (uint32_t k = 0; k < v.n; ++k) any(d.kids[v.a + k], sub);
    } else if (v.t == J_OBJ) {
      Any sub;
      for (uint32_t k = 0; k < v.n; ++k) any(d.kids[v.a + 2 * k + 1], sub);
    }
  }
};

template <class T>
using OMap = std::vector<std::pair<std::string, T>>;

// ------------------------------------------------------------------ the Go types (objects.py decoders)
struct Req {  // ClusterSelectorRequirement
  std::string key, op;
  std::optional<std::vector<std::string>> values;
};
struct Term {  // ClusterSelectorTerm
  std::optional<std::vector<Req>> exprs, fields;
};
struct Selector {
  std::optional<std::vector<Term>> terms;
};
struct PrefTerm {
  int32_t weight = 0;
  Term pref;
};
struct ClusterAffinity {
  std::optional<Selector> required;
  std::optional<std::vector<PrefTerm>> preferred;
};
struct Affinity {
  std::optional<ClusterAffinity> ca;
};
struct Toleration {
  std::string key, op, value, effect;
  std::optional<int64_t> secs;
};
struct Preferences {
  int64_t min = 0;
  std::optional<int64_t> max, weight;
};
struct Placement {
  std::string cluster;
  Preferences prefs;
};
struct AutoMigration {
  std::optional<std::string> pod_unschedulable_for;
  bool keep = false;
};
struct PolicySpec {
  std::string profile, mode;
  bool sticky = false;
  std::optional<OMap<std::string>> selector;
  std::optional<std::vector<Term>> affinity;
  std::optional<std::vector<Toleration>> tolerations;
  std::optional<int64_t> max_clusters;
  std::optional<std::vector<Placement>> placements;
  bool disable_follower = false;
  std::optional<AutoMigration> am;
  std::optional<bool> avoid_disruption;  // ReplicaRescheduling != nil: its AvoidDisruption
};

void dec_strings(Dec& D, uint32_t x, std::optional<std::vector<std::string>>& out) {
  D.slice(x, out, [&](uint32_t e, std::string& s) { D.str(e, s); });
}
void dec_req(Dec& D, uint32_t x, Req& r) {
  static const sv N[] = {"key", "operator", "values"};
  if (D.null(x)) return;
  D.fields(x, N, [&](int f, uint32_t v) {
    if (f == 0) D.str(v, r.key);
    else if (f == 1) D.str(v, r.op);
    else dec_strings(D, v, r.values);
  });
}
void dec_term(Dec& D, uint32_t x, Term& t) {
  static const sv N[] = {"matchExpressions", "matchFields"};
  if (D.null(x)) return;
  D.fields(x, N, [&](int f, uint32_t v) {
    D.slice(v, f == 0 ? t.exprs : t.fields, [&](uint32_t e, Req& r) { dec_req(D, e, r); });
  });
}
void dec_terms(Dec& D, uint32_t x, std::optional<std::vector<Term>>& out) {
  D.slice(x, out, [&](uint32_t e, Term& t) { dec_term(D, e, t); });
}
void dec_selector(Dec& D, uint32_t x, Selector& s) {
  static const sv N[] = {"clusterSelectorTerms"};
  if (D.null(x)) return;
  D.fields(x, N, [&](int, uint32_t v) { dec_terms(D, v, s.terms); });
}
void dec_affinity(Dec& D, uint32_t x, Affinity& a) {
  static const sv NA[] = {"clusterAffinity"};
  static const sv NC[] = {"requiredDuringSchedulingIgnoredDuringExecution", "preferredDuringSchedulingIgnoredDuringExecution"};
  static const sv NP[] = {"weight", "preference"};
  if (D.null(x)) return;
  D.fields(x, NA, [&](int, uint32_t v) {
    if (D.null(v)) {
      a.ca.reset();
      return;
    }
    if (!a.ca) a.ca.emplace();
    ClusterAffinity& ca = *a.ca;
    D.fields(v, NC, [&](int f, uint32_t w) {
      if (f == 0) {
        if (D.null(w)) {
          ca.required.reset();
          return;
        }
        if (!ca.required) ca.required.emplace();
        dec_selector(D, w, *ca.required);
      } else {
        D.slice(w, ca.preferred, [&](uint32_t e, PrefTerm& p) {
          if (D.null(e)) return;
          D.fields(e, NP, [&](int g, uint32_t y) {
            if (g == 0) D.int32(y, p.weight);
            else dec_term(D, y, p.pref);
          });
        });
      }
    });
  });
}
void dec_tolerations(Dec& D, uint32_t x, std::optional<std::vector<Toleration>>& out) {
  static const sv N[] = {"key", "operator", "value", "effect", "tolerationSeconds"};
  D.slice(x, out, [&](uint32_t e, Toleration& t) {
    if (D.null(e)) return;
    D.fields(e, N, [&](int f, uint32_t v) {
      if (f == 0) D.str(v, t.key);
      else if (f == 1) D.str(v, t.op);
      else if (f == 2) D.str(v, t.value);
      else if (f == 3) D.str(v, t.effect);
      else D.ptr_int64(v, t.secs);
    });
  });
}
void dec_placements(Dec& D, uint32_t x, std::optional<std::vector<Placement>>& out) {
  static const sv N[] = {"cluster", "preferences"};
  static const sv NP[] = {"minReplicas", "maxReplicas", "weight"};
  D.slice(x, out, [&](uint32_t e, Placement& p) {
    if (D.null(e)) return;
    D.fields(e, N, [&](int f, uint32_t v) {
      if (f == 0) {
        D.str(v, p.cluster);
      } else if (!D.null(v)) {
        D.fields(v, NP, [&](int g, uint32_t w) {
          if (g == 0) D.int64(w, p.prefs.min);
          else if (g == 1) D.ptr_int64(w, p.prefs.max);
          else D.ptr_int64(w, p.prefs.weight);
        });
      }
    });
  });
}
void dec_string_map(Dec& D, uint32_t x, std::optional<OMap<std::string>>& out) {
  D.map(x, out, [&](uint32_t e, std::string& s) { D.str(e, s); });
}
// POLICY_SPEC (types_propagationpolicy.go:62-110)
void dec_policy_spec(Dec& D, uint32_t x, PolicySpec& s) {
  static const sv N[] = {"schedulingProfile", "schedulingMode", "stickyCluster", "clusterSelector", "clusterAffinity",
                         "tolerations", "maxClusters", "placement", "disableFollowerScheduling", "autoMigration",
                         "replicaRescheduling"};
  static const sv NAM[] = {"when", "keepUnschedulableReplicas"};
  static const sv NW[] = {"podUnschedulableFor"};
  static const sv NRR[] = {"avoidDisruption"};
  if (D.null(x)) return;
  D.fields(x, N, [&](int f, uint32_t v) {
    switch (f) {
      case 0: D.str(v, s.profile); break;
      case 1: D.str(v, s.mode); break;
      case 2: D.boolean(v, s.sticky); break;
      case 3: dec_string_map(D, v, s.selector); break;
      case 4: dec_terms(D, v, s.affinity); break;
      case 5: dec_tolerations(D, v, s.tolerations); break;
      case 6: D.ptr_int64(v, s.max_clusters); break;
      case 7: dec_placements(D, v, s.placements); break;
      case 8: D.boolean(v, s.disable_follower); break;
      case 9:
        if (D.null(v)) {
          s.am.reset();
          break;
        }
        if (!s.am) s.am.emplace();
        D.fields(v, NAM, [&](int g, uint32_t w) {
          if (g == 1) {
            D.boolean(w, s.am->keep);
          } else if (!D.null(w)) {
            D.fields(w, NW, [&](int, uint32_t y) { D.ptr_str(y, s.am->pod_unschedulable_for); });
          }
        });
        break;
      default:
        if (D.null(v)) {
          s.avoid_disruption.reset();
          break;
        }
        if (!s.avoid_disruption) s.avoid_disruption = false;
        D.fields(v, NRR, [&](int, uint32_t w) {
          bool b = *s.avoid_disruption;
          D.boolean(w, b);
          s.avoid_disruption = b;
        });
    }
  });
}

// ------------------------------------------------------------------ the policy table
struct Policy {
  std::string ns, name;
  int64_t generation = 0;  // metadata.generation (the trigger hash's policyGeneration)
  bool ok = false;
  std::string err;
  PolicySpec spec;
};
// PropagationPolicy.from_json: metadata name / namespace, spec decoded (a missing or null spec = {})
void load_policy(sv text, Policy& P) {
  JDoc d;
  uint32_t root;
  if (!parse(text, d, &root) || d.v[root].t != J_OBJ) {
    P.err = "policy: not a JSON object";
    return;
  }
  const int64_t meta = get(d, root, "metadata");
  if (meta >= 0 && d.v[meta].t == J_OBJ) {
    const int64_t nm = get(d, (uint32_t)meta, "name"), ns = get(d, (uint32_t)meta, "namespace");
    if (nm >= 0 && d.v[nm].t == J_STR) P.name.assign(d.str((uint32_t)nm));
    if (ns >= 0 && d.v[ns].t == J_STR) P.ns.assign(d.str((uint32_t)ns));
    const int64_t g = get(d, (uint32_t)meta, "generation");
    if (g >= 0 && d.v[g].t == J_NUM && d.v[g].isint && d.v[g].fits) P.generation = d.v[g].i;
  }
  const int64_t spec = get(d, root, "spec");
  // `d.get("spec") or {}`: null, {}, "" , 0, false and [] all decode as the empty spec
  bool empty = spec < 0;
  if (!empty) {
    const JV& v = d.v[spec];
    empty = v.t == J_NULL || v.t == J_FALSE || (v.t == J_OBJ && v.n == 0) || (v.t == J_ARR && v.n == 0) ||
            (v.t == J_STR && v.n == 0) || (v.t == J_NUM && v.d == 0.0);
  }
  if (empty) {
    P.ok = true;
    return;
  }
  Dec D{d, true};
  dec_policy_spec(D, (uint32_t)spec, P.spec);
  if (D.err) P.err = std::string("policy spec: json: cannot unmarshal into ") + D.err;
  else P.ok = true;
}

// ------------------------------------------------------------------ typed views of the object itself
// (decoded through the unstructured round trip: sorted unique keys)
struct PC {  // PlacementWithController
  std::string controller;
  std::optional<std::vector<std::string>> clusters;
};
// _OBJ_PLACEMENTS: type-checks apiVersion, kind, metadata and spec.placements; the error or null.
// replaced_ann: the metadata.annotations node a trigger annotation replaced (AddAnnotation over annotations
// that are not a string map writes a fresh one), not type-checked
const char* decode_placements_view(const JDoc& d, uint32_t root, std::optional<std::vector<PC>>& pls,
                                   uint32_t replaced_ann = UINT32_MAX) {
  static const sv N[] = {"apiVersion", "kind", "metadata", "spec"};
  static const sv NM[] = {"name", "namespace", "generateName", "uid", "resourceVersion", "generation", "labels", "annotations"};
  static const sv NS[] = {"placements"};
  static const sv NPC[] = {"controller", "placement"};
  static const sv NPL[] = {"clusters"};
  static const sv NCR[] = {"name"};
  Dec D{d, true};
  std::string scratch;
  D.fields(root, N, [&](int f, uint32_t v) {
    if (f <= 1) {
      D.str(v, scratch);
    } else if (f == 2) {
      D.fields(v, NM, [&](int g, uint32_t w) {
        if (g <= 4) {
          D.str(w, scratch);
        } else if (g == 5) {
          int64_t i = 0;
          D.int64(w, i);
        } else if (g == 6 || w != replaced_ann) {
          std::optional<OMap<std::string>> m;
          dec_string_map(D, w, m);
        }
      });
    } else {
      D.fields(v, NS, [&](int, uint32_t w) {
        D.slice(w, pls, [&](uint32_t e, PC& pc) {
          D.fields(e, NPC, [&](int g, uint32_t y) {
            if (g == 0) {
              D.str(y, pc.controller);
            } else {
              D.fields(y, NPL, [&](int, uint32_t z) {
                D.slice(z, pc.clusters, [&](uint32_t q, std::string& s) {
                  D.fields(q, NCR, [&](int, uint32_t r) { D.str(r, s); });
                });
              });
            }
          });
        });
      });
    }
  });
  return D.err;
}
struct Patch {  // OverridePatch; value: interface{} (a node of the object), or a replica count set here
  std::string op, path;
  Dec::Any value;
  uint32_t node = 0;
  bool set = false;  // value = n (written by updateOverridesMap)
  int64_t n = 0;
};
struct CO {
  std::string cluster;
  std::optional<std::vector<Patch>> patches;
};
struct CtrlO {
  std::string controller;
  std::optional<std::vector<CO>> clusters;
};
// _OBJ_OVERRIDES; spec_set: spec decoded to a non-nil pointer
const char* decode_overrides_view(const JDoc& d, uint32_t root, std::optional<std::vector<CtrlO>>& ovs, bool& spec_set) {
  static const sv N[] = {"spec"};
  static const sv NS[] = {"overrides"};
  static const sv NC[] = {"controller", "clusters"};
  static const sv NCO[] = {"clusterName", "paths"};
  static const sv NP[] = {"op", "path", "value"};
  Dec D{d, true};
  D.fields(root, N, [&](int, uint32_t v) {
    if (D.null(v)) {  // *spec = nil (a later case-folded "spec" member may set it again)
      ovs.reset();
      spec_set = false;
      return;
    }
    if (D.at(v).t == J_OBJ) spec_set = true;
    D.fields(v, NS, [&](int, uint32_t w) {
      D.slice(w, ovs, [&](uint32_t e, CtrlO& c) {
        D.fields(e, NC, [&](int g, uint32_t y) {
          if (g == 0) {
            D.str(y, c.controller);
          } else {
            D.slice(y, c.clusters, [&](uint32_t q, CO& co) {
              D.fields(q, NCO, [&](int h, uint32_t r) {
                if (h == 0) {
                  D.str(r, co.cluster);
                } else {
                  D.slice(r, co.patches, [&](uint32_t s, Patch& p) {
                    D.fields(s, NP, [&](int k, uint32_t t) {
                      if (k == 0) {
                        D.str(t, p.op);
                      } else if (k == 1) {
                        D.str(t, p.path);
                      } else {
                        D.any(t, p.value);
                        p.node = t;
                      }
                    });
                  });
                }
              });
            });
          }
        });
      });
    });
  });
  return D.err;
}

// ------------------------------------------------------------------ one object → one SchedulingUnit
struct Unit {  // strings by value; interned in the serial merge
  int status = KAD_OBJ_OK;
  std::string msg;
  int32_t policy = -1;
  std::string ns, name;
  uint32_t flags = 0;
  int64_t desired = 0, max_clusters = 0;
  std::vector<std::pair<std::string, std::string>> sel;
  std::vector<Toleration> tols;
  std::vector<Term> rterms;
  std::vector<PrefTerm> pterms;
  std::vector<std::string> place;  // sorted, unique
  std::vector<std::pair<std::string, std::optional<int64_t>>> cur;
  OMap<int64_t> wt, mn, mx, cap;
};

int64_t f64_to_i64(double x) {  // Go int64(f) on amd64: truncation, NaN / out of range → MinInt64
  if (x != x || !(x >= -9.223372036854776e18 && x < 9.223372036854776e18)) return INT64_MIN;
  return (int64_t)x;
}
// strconv.Atoi on a 64-bit platform
bool atoi64(sv s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '+' || s[0] == '-')) {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  uint64_t v = 0;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') return false;
    const uint64_t dg = (uint64_t)(c - '0');
    if (v > (lim - dg) / 10) return false;
    v = v * 10 + dg;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

struct Builder {
  const kad_type_config& tc;
  const std::vector<Policy>& pols;
  const std::unordered_map<std::string, int32_t>& pol_index;  // namespace + '\0' + name
  std::vector<std::string> replicas_fields;                   // spec.template + the dot path
  std::string replicas_slash;                                 // ToSlashPath(ReplicasSpec)
  bool replicas_empty;                                        // ReplicasSpec == ""

  // metadata.annotations / .labels as GetAnnotations reads them: a string map, else none
  static int64_t string_map(const JDoc& d, uint32_t root, sv field) {
    const int64_t meta = get(d, root, "metadata");
    if (meta < 0 || d.v[meta].t != J_OBJ) return -1;
    const int64_t m = get(d, (uint32_t)meta, field);
    if (m < 0 || d.v[m].t != J_OBJ) return -1;
    const JV& o = d.v[m];
    for (uint32_t k = 0; k < o.n; ++k)
      if (d.v[d.kids[o.a + 2 * k + 1]].t != J_STR) return -1;
    return m;
  }

  // forced >= -1: the caller's policy index (-1 none); -2: MatchedPolicyKey through the labels
  void build(sv text, Unit& u, JDoc& d, JDoc& ad, int32_t forced) {
    uint32_t root;
    if (!parse(text, d, &root) || d.v[root].t != J_OBJ) fail(KAD_OBJ_BAD_JSON, "object: not a JSON object");
    const int64_t labels = string_map(d, root, "labels");
    const int64_t anns = string_map(d, root, "annotations");
    auto ann = [&](sv key) -> std::optional<sv> {
      if (anns < 0) return std::nullopt;
      const int64_t v = get(d, (uint32_t)anns, key);
      if (v < 0) return std::nullopt;
      return d.str((uint32_t)v);
    };
    // MatchedPolicyKey (scheduler/util.go:37-49) and the informer lookup (scheduler.go:359-372)
    if (forced >= -1) {  // the caller's index, range-checked on entry (policy_of_ok)
      if (forced < 0) {
        u.status = KAD_OBJ_NO_POLICY;
        return;
      }
      u.policy = forced;
    } else {
      std::optional<std::string> key;
      const int64_t pl = labels >= 0 ? get(d, (uint32_t)labels, POLICY_LABEL) : -1;
      const int64_t cl = labels >= 0 ? get(d, (uint32_t)labels, CLUSTER_POLICY_LABEL) : -1;
      if (pl >= 0 && tc.namespaced) {
        std::string ns;
        const int64_t meta = get(d, root, "metadata");
        const int64_t nsv = meta >= 0 && d.v[meta].t == J_OBJ ? get(d, (uint32_t)meta, "namespace") : -1;
        if (nsv >= 0 && d.v[nsv].t == J_STR) ns.assign(d.str((uint32_t)nsv));
        key = ns + '\0' + std::string(d.str((uint32_t)pl));
      } else if (cl >= 0) {
        key = std::string(1, '\0') + std::string(d.str((uint32_t)cl));
      }
      if (!key) {
        u.status = KAD_OBJ_NO_POLICY;
        return;
      }
      auto it = pol_index.find(*key);
      if (it == pol_index.end()) {
        u.status = KAD_OBJ_POLICY_NOT_FOUND;
        return;
      }
      u.policy = it->second;
    }
    const Policy& P = pols[(size_t)u.policy];
    if (!P.ok) fail(KAD_OBJ_POLICY_ERROR, P.err);
    const PolicySpec& spec = P.spec;

    // getTemplate (schedulingunit.go:165-179)
    {
      const int64_t sp = get(d, root, "spec");
      if (sp < 0) fail(KAD_OBJ_UNIT_ERROR, "template not found");
      if (d.v[sp].t != J_OBJ) fail(KAD_OBJ_UNIT_ERROR, "error retrieving template: .spec accessor error");
      const int64_t t = get(d, (uint32_t)sp, "template");
      if (t < 0) fail(KAD_OBJ_UNIT_ERROR, "template not found");
      if (d.v[t].t != J_OBJ) fail(KAD_OBJ_UNIT_ERROR, "error retrieving template: .spec.template accessor error: not a map");
      const uint32_t tm = (uint32_t)t;
      for (sv k : {sv("apiVersion"), sv("kind")}) {
        const int64_t x = get(d, tm, k);
        if (x >= 0 && d.v[x].t != J_NULL && d.v[x].t != J_STR) fail(KAD_OBJ_UNIT_ERROR, "template cannot be converted from unstructured");
      }
      const int64_t meta = get(d, tm, "metadata");
      if (meta >= 0 && d.v[meta].t != J_NULL) {
        if (d.v[meta].t != J_OBJ) fail(KAD_OBJ_UNIT_ERROR, "template cannot be converted from unstructured");
        const uint32_t m = (uint32_t)meta;
        for (sv k : {sv("name"), sv("namespace"), sv("generateName")}) {
          const int64_t x = get(d, m, k);
          if (x >= 0 && d.v[x].t != J_NULL && d.v[x].t != J_STR) fail(KAD_OBJ_UNIT_ERROR, "template cannot be converted from unstructured");
          if (x >= 0 && d.v[x].t == J_STR) {
            if (k == "name") u.name.assign(d.str((uint32_t)x));
            else if (k == "namespace") u.ns.assign(d.str((uint32_t)x));
          }
        }
        for (sv k : {sv("labels"), sv("annotations")}) {
          const int64_t x = get(d, m, k);
          if (x < 0 || d.v[x].t == J_NULL) continue;
          if (d.v[x].t != J_OBJ) fail(KAD_OBJ_UNIT_ERROR, "template cannot be converted from unstructured");
          const JV& o = d.v[x];
          for (uint32_t q = 0; q < o.n; ++q)
            if (d.v[d.kids[o.a + 2 * q + 1]].t != J_STR) fail(KAD_OBJ_UNIT_ERROR, "template cannot be converted from unstructured");
        }
      }
    }

    // scheduling mode (:224-259) and DesiredReplicas (:48-58, GetInt64FromPath)
    sv mode = (spec.mode == DUPLICATE || spec.mode == DIVIDE) ? sv(spec.mode) : DUPLICATE;
    if (auto m = ann(SCHEDULING_MODE_ANN); m && (*m == DUPLICATE || *m == DIVIDE)) mode = *m;
    if (mode == DIVIDE && replicas_empty) mode = DUPLICATE;  // ReplicasSpec == ""
    if (mode == DIVIDE) {
      uint32_t x = root;
      bool found = true;
      for (const std::string& f : replicas_fields) {
        if (d.v[x].t != J_OBJ) fail(KAD_OBJ_UNIT_ERROR, "cannot access [spec template]: accessor error: not a map");
        const int64_t y = get(d, x, f);
        if (y < 0) {
          found = false;
          break;
        }
        x = (uint32_t)y;
      }
      if (found) {
        const JV& v = d.v[x];
        if (v.t != J_NUM || !v.isint || !v.fits) fail(KAD_OBJ_UNIT_ERROR, "cannot access [spec template]: expected int64");
        u.flags |= KAD_SU_HAS_DESIRED;
        u.desired = v.i;
      }
    }

    current_replicas(d, root, u);

    u.flags |= KAD_SU_AVOID_DISRUPTION;
    if (spec.am) {  // :91-100, getAutoMigrationInfo :261-272
      u.flags |= KAD_SU_HAS_AUTO_MIGRATION;
      if (spec.am->keep) u.flags |= KAD_SU_KEEP_UNSCHED;
      if (auto v = ann(AUTO_MIGRATION_INFO_ANN)) {
        JDoc& a = ad;
        uint32_t r;
        if (!parse(*v, a, &r)) fail(KAD_OBJ_UNIT_ERROR, "auto-migration-info: invalid JSON");
        Dec D{a, false};
        std::optional<OMap<int64_t>> ec;
        static const sv N[] = {"estimatedCapacity"};
        if (!D.null(r))
          D.fields(r, N, [&](int, uint32_t x) { D.map(x, ec, [&](uint32_t e, int64_t& i) { D.int64(e, i); }); });
        if (D.err) fail(KAD_OBJ_UNIT_ERROR, std::string("auto-migration-info: json: cannot unmarshal into ") + D.err);
        if (ec) u.cap = std::move(*ec);
      }
    }
    if (spec.avoid_disruption && !*spec.avoid_disruption) u.flags &= ~KAD_SU_AVOID_DISRUPTION;
    if (mode == DUPLICATE) u.flags |= KAD_SU_DUPLICATE;

    bool sticky = spec.sticky;  // :278-304
    if (auto v = ann(STICKY_ANN)) {
      if (*v == "true") sticky = true;
      else if (*v == "false") sticky = false;
    }
    if (sticky) u.flags |= KAD_SU_STICKY;

    // ClusterSelector (:306-334): the annotation replaces the policy's when it decodes
    const std::optional<OMap<std::string>>* selp = &spec.selector;
    std::optional<OMap<std::string>> sel_ann;
    if (auto v = ann(SELECTOR_ANN)) {
      JDoc& a = ad;
      uint32_t r;
      if (parse(*v, a, &r)) {
        Dec D{a, false};
        dec_string_map(D, r, sel_ann);
        if (!D.err) selp = &sel_ann;
      }
    }
    if (*selp) u.sel = **selp;

    // placements (:450-668): the annotation's list, else the policy's
    std::optional<std::vector<Placement>> ann_pl;
    bool have_ann_pl = false;
    if (auto v = ann(PLACEMENTS_ANN)) {
      JDoc& a = ad;
      uint32_t r;
      if (parse(*v, a, &r)) {
        Dec D{a, false};
        dec_placements(D, r, ann_pl);
        if (!D.err) {
          have_ann_pl = true;
          if (!ann_pl) ann_pl.emplace();  // "null": an empty list
        }
      }
    }
    const std::vector<Placement>* pols_pl = spec.placements ? &*spec.placements : nullptr;
    const std::vector<Placement>* names_from = have_ann_pl ? &*ann_pl : pols_pl;
    if (names_from) {
      for (const Placement& p : *names_from) u.place.push_back(p.cluster);
      std::sort(u.place.begin(), u.place.end());
      u.place.erase(std::unique(u.place.begin(), u.place.end()), u.place.end());
    }
    auto pref_map = [&](const std::vector<Placement>& pl, int which, OMap<int64_t>& out) {
      out.clear();
      std::unordered_map<std::string, size_t> pos;  // (long lists only)
      for (const Placement& p : pl) {
        int64_t v;
        if (which == 0) v = p.prefs.min;
        else if (which == 1) {
          if (!p.prefs.max) continue;
          v = *p.prefs.max;
        } else {
          if (!p.prefs.weight) continue;
          v = *p.prefs.weight;
        }
        size_t at = SIZE_MAX;
        if (pl.size() <= 16) {
          for (size_t q = 0; q < out.size() && at == SIZE_MAX; ++q)
            if (out[q].first == p.cluster) at = q;
        } else if (auto it = pos.find(p.cluster); it != pos.end()) {
          at = it->second;
        }
        if (at != SIZE_MAX) {
          out[at].second = v;
        } else {
          if (pl.size() > 16) pos.emplace(p.cluster, out.size());
          out.emplace_back(p.cluster, v);
        }
      }
    };
    for (int which = 0; which < 3; ++which) {
      OMap<int64_t>& dst = which == 0 ? u.mn : (which == 1 ? u.mx : u.wt);
      if (pols_pl) pref_map(*pols_pl, which, dst);
      if (have_ann_pl) {
        OMap<int64_t> m;
        pref_map(*ann_pl, which, m);
        bool ok = true;
        for (const auto& kv : m) ok = ok && kv.second >= 0;
        if (ok) dst = std::move(m);  // negative values invalidate the override (:510-624)
      }
    }

    // Affinity (:336-377)
    std::optional<Affinity> aff;
    if (spec.affinity && !spec.affinity->empty()) {
      aff.emplace();
      aff->ca.emplace();
      aff->ca->required.emplace();
      aff->ca->required->terms = *spec.affinity;
    }
    if (auto v = ann(AFFINITY_ANN)) {
      JDoc& a = ad;
      uint32_t r;
      if (parse(*v, a, &r)) {
        Dec D{a, false};
        std::optional<Affinity> x;
        if (!D.null(r)) {
          x.emplace();
          dec_affinity(D, r, *x);
        }
        if (!D.err) aff = std::move(x);
      }
    }
    if (aff && aff->ca) {
      u.flags |= KAD_SU_HAS_CLUSTER_AFFINITY;
      const ClusterAffinity& ca = *aff->ca;
      if (ca.required) {
        u.flags |= KAD_SU_HAS_REQUIRED;
        if (ca.required->terms) u.rterms = *ca.required->terms;
      }
      if (ca.preferred) u.pterms = *ca.preferred;
    }

    // Tolerations (:379-407): "null" decodes to none
    const std::optional<std::vector<Toleration>>* tolp = &spec.tolerations;
    std::optional<std::vector<Toleration>> tol_ann;
    if (auto v = ann(TOLERATIONS_ANN)) {
      JDoc& a = ad;
      uint32_t r;
      if (parse(*v, a, &r)) {
        Dec D{a, false};
        dec_tolerations(D, r, tol_ann);
        if (!D.err) tolp = &tol_ann;
      }
    }
    if (*tolp) u.tols = **tolp;

    // MaxClusters (:409-448)
    std::optional<int64_t> mc = spec.max_clusters;
    if (auto v = ann(MAX_CLUSTERS_ANN)) {
      int64_t n;
      if (atoi64(*v, &n) && n >= 0) mc = n;
    }
    if (mc) {
      u.flags |= KAD_SU_HAS_MAX_CLUSTERS;
      u.max_clusters = *mc;
    }
  }

  // getCurrentReplicasFromObject (schedulingunit.go:181-222): the global scheduler's placement and its
  // replica overrides (util.GetOverrides, util/overrides.go:68-112)
  void current_replicas(const JDoc& d, uint32_t root, Unit& u) {
    std::optional<std::vector<std::string>> names;
    {
      std::optional<std::vector<PC>> pls;
      if (const char* e = decode_placements_view(d, root, pls))
        fail(KAD_OBJ_UNIT_ERROR, std::string("placements: json: cannot unmarshal into ") + e);
      if (pls)
        for (const PC& pc : *pls)
          if (pc.controller == PREFIXED_GLOBAL_SCHEDULER) {
            if (pc.clusters) names = pc.clusters;
            break;
          }
    }
    std::optional<std::vector<CtrlO>> ovs;
    bool spec_set = false;
    const char* oerr = decode_overrides_view(d, root, ovs, spec_set);
    if (oerr) fail(KAD_OBJ_UNIT_ERROR, std::string("overrides: json: cannot unmarshal into ") + oerr);
    const std::vector<CO>* clusters = nullptr;
    if (ovs)
      for (const CtrlO& c : *ovs)
        if (c.controller == PREFIXED_GLOBAL_SCHEDULER) {
          if (c.clusters) clusters = &*c.clusters;
          break;
        }
    std::unordered_map<std::string, const std::vector<Patch>*> by_cluster;
    if (clusters) {
      for (const CO& co : *clusters) {
        if (by_cluster.count(co.cluster)) fail(KAD_OBJ_UNIT_ERROR, "cluster \"" + co.cluster + "\" appears more than once");
        if (co.patches)
          for (const Patch& p : *co.patches)
            if (p.path == "/metadata/namespace" || p.path == "/metadata/name" || p.path == "/metadata/generateName" ||
                p.path == "/kind")
              fail(KAD_OBJ_UNIT_ERROR, "override for cluster \"" + co.cluster + "\" has an invalid path: " + p.path);
        by_cluster.emplace(co.cluster, co.patches ? &*co.patches : nullptr);
      }
    }
    if (!names) return;
    std::vector<std::string> uniq;
    {
      std::unordered_map<std::string, int> seen;
      for (const std::string& n : *names)
        if (seen.emplace(n, 1).second) uniq.push_back(n);
    }
    for (const std::string& n : uniq) {
      std::optional<int64_t> rep;
      auto it = by_cluster.find(n);
      if (it != by_cluster.end() && it->second)
        for (const Patch& p : *it->second)
          if (p.path == replicas_slash && (p.op == "replace" || p.op.empty())) {
            if (p.value.t != J_NUM) fail(KAD_OBJ_UNIT_PANIC, "interface conversion: interface {} is not float64");
            rep = f64_to_i64(p.value.f);
            break;
          }
      u.cur.emplace_back(n, rep);
    }
  }
};


// ------------------------------------------------------------------ f3: applySchedulingResult
// A mutable copy of the object (the unstructured map: unique keys, the last member wins) that the result is
// written into, then re-marshalled the way the reference's Update sends it (json.Marshal of the map: keys
// sorted, Go's string escaping and float64 formatting).
struct MV {
  JT t = J_NULL;
  bool isint = false, fits = false;  // number: an integer literal within int64 (an unstructured int64)
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<std::pair<std::string, MV>> o;
  std::vector<MV> a;

  MV* get(sv key) {
    for (auto& kv : o)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
  void set(sv key, MV v) {
    if (MV* x = get(key)) *x = std::move(v);
    else o.emplace_back(std::string(key), std::move(v));
  }
  void erase(sv key) {
    for (size_t k = 0; k < o.size(); ++k)
      if (o[k].first == key) {
        o.erase(o.begin() + (long)k);
        return;
      }
  }
  static MV str(sv x) {
    MV m;
    m.t = J_STR;
    m.s.assign(x);
    return m;
  }
  static MV obj() {
    MV m;
    m.t = J_OBJ;
    return m;
  }
  static MV arr() {
    MV m;
    m.t = J_ARR;
    return m;
  }
  static MV f64(double x) {
    MV m;
    m.t = J_NUM;
    m.d = x;
    return m;
  }
};
// the node as Go holds it: floats_only — an interface{} value decoded by json.Unmarshal (every number a float64)
MV mv_of(const JDoc& d, uint32_t x, bool floats_only) {
  const JV& v = d.v[x];
  MV m;
  m.t = v.t;
  if (v.t == J_NUM) {
    m.isint = v.isint && !floats_only;
    m.fits = v.fits;
    m.i = v.i;
    m.d = v.d;
  } else if (v.t == J_STR) {
    m.s.assign(d.str(x));
  } else if (v.t == J_ARR) {
    m.a.reserve(v.n);
    for (uint32_t k = 0; k < v.n; ++k) m.a.push_back(mv_of(d, d.kids[v.a + k], floats_only));
  } else if (v.t == J_OBJ) {
    for (uint32_t k = 0; k < v.n; ++k) m.set(d.str(d.kids[v.a + 2 * k]), mv_of(d, d.kids[v.a + 2 * k + 1], floats_only));
  }
  return m;
}

// encodeState.string (Go 1.19, HTML escaping on); gojson._enc_str
void emit_str(sv s, std::string& out) {
  static const char* hex = "0123456789abcdef";
  out += '"';
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      if (c == '"') out += "\\\"";
      else if (c == '\\') out += "\\\\";
      else if (c >= 0x20 && c != '<' && c != '>' && c != '&') out += (char)c;
      else if (c == '\n') out += "\\n";
      else if (c == '\r') out += "\\r";
      else if (c == '\t') out += "\\t";
      else {
        out += "\\u00";
        out += hex[c >> 4];
        out += hex[c & 0xF];
      }
      ++i;
      continue;
    }
    // one UTF-8 sequence (the parser only produces valid ones); U+2028 / U+2029 escaped
    const size_t n = c >= 0xF0 ? 4 : (c >= 0xE0 ? 3 : 2);
    if (n == 3 && c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
        ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      out += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
    } else {
      out.append(s.data() + i, std::min(n, s.size() - i));
    }
    i += n;
  }
  out += '"';
}
// floatEncoder (encoding/json/encode.go): 'f' unless the magnitude is < 1e-6 or >= 1e21, shortest digits
void emit_f64(double f, std::string& out) {
  char buf[64];
  const double ab = std::fabs(f);
  const bool e = ab != 0 && (ab < 1e-6 || ab >= 1e21);
  auto r = std::to_chars(buf, buf + sizeof buf, f, e ? std::chars_format::scientific : std::chars_format::fixed);
  std::string t(buf, r.ptr);
  if (e) {  // e-07 → e-7
    const size_t n = t.size();
    if (n >= 4 && t[n - 4] == 'e' && t[n - 3] == '-' && t[n - 2] == '0') t.erase(n - 2, 1);
  }
  out += t;
}
void emit(const MV& m, std::string& out) {
  switch (m.t) {
    case J_NULL: out += "null"; break;
    case J_TRUE: out += "true"; break;
    case J_FALSE: out += "false"; break;
    case J_STR: emit_str(m.s, out); break;
    case J_NUM:
      if (m.isint && m.fits) out += std::to_string(m.i);
      else if (!std::isfinite(m.d)) fail(KAD_APPLY_BAD_JSON, "object: a number out of float64 range");  // Go rejects it
      else emit_f64(m.d, out);
      break;
    case J_ARR:
      out += '[';
      for (size_t k = 0; k < m.a.size(); ++k) {
        if (k) out += ',';
        emit(m.a[k], out);
      }
      out += ']';
      break;
    case J_OBJ: {
      std::vector<const std::pair<std::string, MV>*> ks;
      ks.reserve(m.o.size());
      for (const auto& kv : m.o) ks.push_back(&kv);
      std::sort(ks.begin(), ks.end(), [](auto* x, auto* y) { return x->first < y->first; });
      out += '{';
      for (size_t k = 0; k < ks.size(); ++k) {
        if (k) out += ',';
        emit_str(ks[k]->first, out);
        out += ':';
        emit(ks[k]->second, out);
      }
      out += '}';
    }
  }
}

// unstructured.SetNestedField(obj, value, a, b): a created when missing, an error when it is not a map
void set_nested(MV& root, sv a, sv b, MV value) {
  MV* x = root.get(a);
  if (!x) {
    root.set(a, MV::obj());
    x = root.get(a);
  } else if (x->t != J_OBJ) {
    fail(KAD_APPLY_ERROR, std::string("value cannot be set because ") + std::string(a) + " is not a map[string]interface{}");
  }
  x->set(b, std::move(value));
}

// time.Duration.String
std::string duration_string(int64_t d) {
  if (d == 0) return "0s";
  const bool neg = d < 0;
  uint64_t u = neg ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;
  auto frac = [](uint64_t v, int prec, std::string& fs) {
    std::string digits;
    bool printed = false;
    for (int k = 0; k < prec; ++k) {
      const int dg = (int)(v % 10);
      printed = printed || dg != 0;
      if (printed) digits += (char)('0' + dg);
      v /= 10;
    }
    std::reverse(digits.begin(), digits.end());
    fs = printed ? "." + digits : "";
    return v;
  };
  std::string s, fs;
  if (u < 1000000000ull) {
    if (u < 1000) {
      s = std::to_string(u) + "ns";
    } else if (u < 1000000) {
      const uint64_t w = frac(u, 3, fs);
      s = std::to_string(w) + fs + "\xC2\xB5s";
    } else {
      const uint64_t w = frac(u, 6, fs);
      s = std::to_string(w) + fs + "ms";
    }
  } else {
    uint64_t w = frac(u, 9, fs);
    s = std::to_string(w % 60) + fs + "s";
    w /= 60;
    if (w > 0) {
      s = std::to_string(w % 60) + "m" + s;
      w /= 60;
      if (w > 0) s = std::to_string(w) + "h" + s;
    }
  }
  return neg ? "-" + s : s;
}

struct Applier {
  const kad_type_config& tc;
  std::string replicas_slash;  // ToSlashPath(ReplicasSpec)

  MV patch_json(const JDoc& d, const Patch& p) {  // the typed patch, marshalled (value: float64 after the round trip)
    MV m = MV::obj();
    if (!p.op.empty()) m.set("op", MV::str(p.op));
    m.set("path", MV::str(p.path));
    if (p.set) m.set("value", MV::f64((double)p.n));
    else if (p.value.t != J_NULL) m.set("value", mv_of(d, p.node, true));
    return m;
  }

  // applySchedulingResult (scheduler.go:632-695) on the parsed object; true if anything changed
  // the fields apply() wrote (bit 0 spec.placements, 1 spec.overrides, 2 metadata.annotations)
  static constexpr int N_DELTA = 3;
  // trigger: the scheduling-trigger-hash annotation to add first (annotation.AddAnnotation, util/annotation/
  // annotation.go:70-97), as the reconcile does before it schedules; trig_changed: it changed the object (not
  // part of the returned applySchedulingResult flag); ann_only: only that (no result to apply)
  bool apply(const JDoc& d, uint32_t root, MV& obj, uint32_t& wrote, const std::vector<std::string>& clusters,
             const OMap<int64_t>& desired, bool follower, std::optional<int64_t> threshold,
             std::optional<sv> trigger, bool ann_only, bool& trig_changed) {
    trig_changed = false;
    bool modified = false;
    bool spec_created = false;
    if (ann_only) goto annotations;
    // util.SetPlacementClusterNames (util/placement.go:44-59)
    {
      std::optional<std::vector<PC>> po;
      uint32_t replaced = UINT32_MAX;
      if (trigger) {
        const int64_t meta = get(d, root, "metadata");
        const int64_t an = meta >= 0 && d.v[meta].t == J_OBJ ? get(d, (uint32_t)meta, "annotations") : -1;
        if (an >= 0) replaced = (uint32_t)an;
      }
      if (const char* e = decode_placements_view(d, root, po, replaced))
        fail(KAD_APPLY_ERROR, std::string("placements: ") + e);
      std::vector<PC> pls = po ? *po : std::vector<PC>();
      int idx = -1;
      for (size_t k = 0; k < pls.size() && idx < 0; ++k)
        if (pls[k].controller == PREFIXED_GLOBAL_SCHEDULER) idx = (int)k;
      bool write = false;
      if (clusters.empty()) {
        if (idx >= 0) {
          pls.erase(pls.begin() + idx);
          write = true;
        }
      } else {
        if (idx < 0) {
          pls.push_back(PC{std::string(PREFIXED_GLOBAL_SCHEDULER), std::nullopt});
          idx = (int)pls.size() - 1;
        }
        std::vector<std::string> old = pls[(size_t)idx].clusters ? *pls[(size_t)idx].clusters : std::vector<std::string>();
        std::sort(old.begin(), old.end());
        old.erase(std::unique(old.begin(), old.end()), old.end());
        if (old != clusters) {  // clusters: sorted, unique
          pls[(size_t)idx].clusters = clusters;
          write = true;
        }
      }
      if (write) {
        MV value;
        if (po || !pls.empty()) {
          value = MV::arr();
          for (const PC& pc : pls) {
            MV e = MV::obj();
            e.set("controller", MV::str(pc.controller));
            MV pl = MV::obj();
            if (pc.clusters && !pc.clusters->empty()) {
              MV cs = MV::arr();
              for (const std::string& n : *pc.clusters) {
                MV c = MV::obj();
                c.set("name", MV::str(n));
                cs.a.push_back(std::move(c));
              }
              pl.set("clusters", std::move(cs));
            }
            e.set("placement", std::move(pl));
            value.a.push_back(std::move(e));
          }
        }
        spec_created = obj.get("spec") == nullptr;
        set_nested(obj, "spec", "placements", std::move(value));
        wrote |= 1u;
        modified = true;
      }
    }
    // UpdateReplicasOverride (scheduler/util.go:71-94)
    {
      std::optional<std::vector<CtrlO>> ovs;
      bool spec_set = false;
      if (const char* e = decode_overrides_view(d, root, ovs, spec_set))
        fail(KAD_APPLY_ERROR, std::string("Error reading cluster overrides: ") + e);
      // util.GetOverrides: the controller's clusters, by name, in list order
      OMap<std::optional<std::vector<Patch>>> ov;
      if (ovs)
        for (const CtrlO& c : *ovs)
          if (c.controller == PREFIXED_GLOBAL_SCHEDULER) {
            if (c.clusters)
              for (const CO& co : *c.clusters) {
                for (const auto& kv : ov)
                  if (kv.first == co.cluster) fail(KAD_APPLY_ERROR, "Error reading cluster overrides: cluster \"" + co.cluster + "\" appears more than once");
                if (co.patches)
                  for (const Patch& p : *co.patches)
                    if (p.path == "/metadata/namespace" || p.path == "/metadata/name" ||
                        p.path == "/metadata/generateName" || p.path == "/kind")
                      fail(KAD_APPLY_ERROR, "Error reading cluster overrides: invalid path " + p.path);
                ov.emplace_back(co.cluster, co.patches);
              }
            break;
          }
      auto desired_of = [&](const std::string& c) -> const int64_t* {
        for (const auto& kv : desired)
          if (kv.first == c) return &kv.second;
        return nullptr;
      };
      // OverrideUpdateNeeded (:154-185)
      bool needed = false;
      size_t checked = 0;
      for (const auto& [cluster, patches] : ov) {
        if (!patches || needed) continue;
        for (const Patch& p : *patches) {
          if (p.path != replicas_slash) continue;
          const int64_t* want = desired_of(cluster);
          if (p.value.t != J_NUM || !want || f64_to_i64(p.value.f) != *want) {
            needed = true;
            break;
          }
          ++checked;
        }
      }
      if (!needed) needed = checked != desired.size();
      if (needed) {
        // updateOverridesMap (:109-152)
        for (size_t k = 0; k < ov.size();) {
          auto& [cluster, patches] = ov[k];
          if (desired_of(cluster) || !patches) {
            ++k;
            continue;
          }
          bool erased = false;
          for (size_t q = 0; q < patches->size(); ++q)
            if ((*patches)[q].path == replicas_slash) {
              patches->erase(patches->begin() + (long)q);
              if (patches->empty()) {
                ov.erase(ov.begin() + (long)k);
                erased = true;
              }
              break;
            }
          if (!erased) ++k;
        }
        for (const auto& [cluster, n] : desired) {
          auto* slot = (std::optional<std::vector<Patch>>*)nullptr;
          for (auto& kv : ov)
            if (kv.first == cluster) slot = &kv.second;
          bool found = false;
          if (slot && *slot)
            for (Patch& p : **slot)
              if (p.path == replicas_slash) {
                p.set = true;
                p.n = n;
                found = true;
                break;
              }
          if (!found) {
            Patch np;
            np.path = replicas_slash;
            np.set = true;
            np.n = n;
            if (slot) {
              if (!*slot) slot->emplace();
              (*slot)->push_back(std::move(np));
            } else {
              ov.emplace_back(cluster, std::vector<Patch>{std::move(np)});
            }
          }
        }
        // util.SetOverrides (util/overrides.go:114-169)
        OMap<std::vector<Patch>> keep;
        for (auto& kv : ov)
          if (kv.second && !kv.second->empty()) keep.emplace_back(kv.first, std::move(*kv.second));
        if (!spec_set && !spec_created) fail(KAD_APPLY_PANIC, "invalid memory address or nil pointer dereference");
        std::optional<std::vector<CtrlO>> cos = ovs;  // the object's overrides (SetOverrides re-reads them)
        int idx = -1;
        if (cos)
          for (size_t k = 0; k < cos->size() && idx < 0; ++k)
            if ((*cos)[k].controller == PREFIXED_GLOBAL_SCHEDULER) idx = (int)k;
        if (keep.empty()) {
          if (idx >= 0) cos->erase(cos->begin() + idx);
        } else {
          if (idx < 0) {
            if (!cos) cos.emplace();
            cos->push_back(CtrlO{std::string(PREFIXED_GLOBAL_SCHEDULER), std::nullopt});
            idx = (int)cos->size() - 1;
          }
          std::sort(keep.begin(), keep.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
          std::vector<CO> cl;
          for (auto& kv : keep) cl.push_back(CO{kv.first, std::move(kv.second)});
          (*cos)[(size_t)idx].clusters = std::move(cl);
        }
        MV value;
        if (cos) {
          value = MV::arr();
          for (const CtrlO& co : *cos) {
            MV e = MV::obj();
            e.set("controller", MV::str(co.controller));
            MV cs;
            if (co.clusters) {
              cs = MV::arr();
              for (const CO& c : *co.clusters) {
                MV x = MV::obj();
                x.set("clusterName", MV::str(c.cluster));
                if (c.patches && !c.patches->empty()) {
                  MV ps = MV::arr();
                  for (const Patch& p : *c.patches) ps.a.push_back(patch_json(d, p));
                  x.set("paths", std::move(ps));
                }
                cs.a.push_back(std::move(x));
              }
            }
            e.set("clusters", std::move(cs));
            value.a.push_back(std::move(e));
          }
        }
        set_nested(obj, "spec", "overrides", std::move(value));
        wrote |= 2u;
        modified = true;
      }
    }
    // the follower-scheduling and pod-unschedulable-threshold annotations (:660-690)
  annotations: {
      OMap<std::string> ann;
      const int64_t am = Builder::string_map(d, root, "annotations");
      if (am >= 0) {
        const JV& o = d.v[am];
        for (uint32_t k = 0; k < o.n; ++k) {
          const sv key = d.str(d.kids[o.a + 2 * k]), val = d.str(d.kids[o.a + 2 * k + 1]);
          bool found = false;
          for (auto& kv : ann)
            if (kv.first == key) {
              kv.second.assign(val);
              found = true;
            }
          if (!found) ann.emplace_back(std::string(key), std::string(val));
        }
      }
      auto find = [&](sv key) -> std::string* {
        for (auto& kv : ann)
          if (kv.first == key) return &kv.second;
        return nullptr;
      };
      bool changed = false;
      if (trigger) {  // AddAnnotation: changed unless the string-map view already holds the value
        std::string* x = find(TRIGGER_HASH_ANN);
        if (am < 0 || !x || *x != *trigger) {
          if ((x = find(TRIGGER_HASH_ANN))) x->assign(*trigger);
          else ann.emplace_back(std::string(TRIGGER_HASH_ANN), std::string(*trigger));
          trig_changed = true;
        }
      }
      if (ann_only) {
        if (trig_changed) {
          MV m = MV::obj();
          for (const auto& kv : ann) m.set(kv.first, MV::str(kv.second));
          set_nested(obj, "metadata", "annotations", std::move(m));
          wrote |= 4u;
          modified = true;
        }
        return false;
      }
      const std::string fv = follower ? "true" : "false";
      if (std::string* x = find(ENABLE_FOLLOWER_ANN); !x || *x != fv) {
        if (x) *x = fv;
        else ann.emplace_back(std::string(ENABLE_FOLLOWER_ANN), fv);
        changed = true;
      }
      if (!threshold) {
        for (size_t k = 0; k < ann.size(); ++k)
          if (ann[k].first == POD_UNSCHEDULABLE_THRESHOLD_ANN) {
            ann.erase(ann.begin() + (long)k);
            changed = true;
            break;
          }
      } else {
        const std::string ds = duration_string(*threshold);
        if (std::string* x = find(POD_UNSCHEDULABLE_THRESHOLD_ANN); !x || *x != ds) {
          if (x) *x = ds;
          else ann.emplace_back(std::string(POD_UNSCHEDULABLE_THRESHOLD_ANN), ds);
          changed = true;
        }
      }
      if (changed || trig_changed) {
        MV m = MV::obj();
        for (const auto& kv : ann) m.set(kv.first, MV::str(kv.second));
        set_nested(obj, "metadata", "annotations", std::move(m));
        wrote |= 4u;
        modified = modified || changed;
      }
    }
    return modified;
  }
};

template <class F>
void parallel_for(int n, int threads, F f, int grain) {
  if (n <= 0) return;
  if (threads <= 1 || n < 2 * grain) {
    f(0, n);
    return;
  }
  const int T = std::min(threads, (n + grain - 1) / grain);
  kadpool::pool().run(T, [&](int t) { f((int)((int64_t)n * t / T), (int)((int64_t)n * (t + 1) / T)); });
}

struct Interner {
  std::unordered_map<std::string, int32_t> ids;
  std::vector<int64_t> off{0};
  std::vector<uint8_t> bytes;
  int32_t id(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    const int32_t i = (int32_t)ids.size();
    ids.emplace(s, i);
    bytes.insert(bytes.end(), s.begin(), s.end());
    off.push_back((int64_t)bytes.size());
    return i;
  }
};

}  // namespace

struct kad_units {
  std::vector<int32_t> status, unit_index, policy_index;
  std::vector<std::string> msg;
  Interner st;
  int32_t n_units = 0;
  std::vector<int32_t> group, version, kind, ns, name;
  std::vector<uint32_t> flags;
  std::vector<int64_t> desired, max_clusters, req_cpu, req_mem, req_eph;
  std::vector<int32_t> scalar_off{0}, scalar_name;
  std::vector<int64_t> scalar_val;
  std::vector<int32_t> tol_off{0}, tol_key, tol_op, tol_value, tol_effect;
  std::vector<int32_t> sel_off{0}, sel_key, sel_value;
  std::vector<int32_t> rq_key, rq_op, rq_val_off{0}, rq_val;
  std::vector<int32_t> rterm_off{0}, rt_req, rt_n_expr, rt_n_field;
  std::vector<int32_t> pterm_off{0}, pt_weight, pt_req, pt_n_expr;
  std::vector<int32_t> place_off{0}, place_name;
  std::vector<int32_t> cur_off{0}, cur_name;
  std::vector<int64_t> cur_rep;
  std::vector<uint8_t> cur_has_rep;
  std::vector<int32_t> wt_off{0}, wt_name, min_off{0}, min_name, max_off{0}, max_name, cap_off{0}, cap_name;
  std::vector<int64_t> wt_val, min_val, max_val, cap_val;
};

namespace {

void merge(kad_units& R, const kad_type_config& tc, std::vector<Unit>& units) {
  Interner& S = R.st;
  const int32_t g = S.id(tc.group ? tc.group : ""), v = S.id(tc.version ? tc.version : ""),
                k = S.id(tc.kind ? tc.kind : "");
  auto add_req = [&](const Req& r) {
    R.rq_key.push_back(S.id(r.key));
    R.rq_op.push_back(S.id(r.op));
    if (r.values)
      for (const std::string& x : *r.values) R.rq_val.push_back(S.id(x));
    R.rq_val_off.push_back((int32_t)R.rq_val.size());
  };
  for (size_t i = 0; i < units.size(); ++i) {
    Unit& u = units[i];
    R.status[i] = u.status;
    R.policy_index[i] = u.policy;
    R.msg[i] = std::move(u.msg);
    if (u.status != KAD_OBJ_OK) continue;
    R.unit_index[i] = R.n_units++;
    R.group.push_back(g);
    R.version.push_back(v);
    R.kind.push_back(k);
    R.ns.push_back(S.id(u.ns));
    R.name.push_back(S.id(u.name));
    R.flags.push_back(u.flags);
    R.desired.push_back(u.desired);
    R.max_clusters.push_back(u.max_clusters);
    R.req_cpu.push_back(0);  // schedulingUnitForFedObject leaves ResourceRequest zero
    R.req_mem.push_back(0);
    R.req_eph.push_back(0);
    R.scalar_off.push_back((int32_t)R.scalar_name.size());
    for (const Toleration& t : u.tols) {
      R.tol_key.push_back(S.id(t.key));
      R.tol_op.push_back(S.id(t.op));
      R.tol_value.push_back(S.id(t.value));
      R.tol_effect.push_back(S.id(t.effect));
    }
    R.tol_off.push_back((int32_t)R.tol_key.size());
    for (const auto& kv : u.sel) {
      R.sel_key.push_back(S.id(kv.first));
      R.sel_value.push_back(S.id(kv.second));
    }
    R.sel_off.push_back((int32_t)R.sel_key.size());
    for (const Term& t : u.rterms) {
      R.rt_req.push_back((int32_t)R.rq_key.size());
      R.rt_n_expr.push_back(t.exprs ? (int32_t)t.exprs->size() : 0);
      R.rt_n_field.push_back(t.fields ? (int32_t)t.fields->size() : 0);
      if (t.exprs)
        for (const Req& r : *t.exprs) add_req(r);
      if (t.fields)
        for (const Req& r : *t.fields) add_req(r);
    }
    R.rterm_off.push_back((int32_t)R.rt_req.size());
    for (const PrefTerm& p : u.pterms) {
      R.pt_weight.push_back(p.weight);
      R.pt_req.push_back((int32_t)R.rq_key.size());
      R.pt_n_expr.push_back(p.pref.exprs ? (int32_t)p.pref.exprs->size() : 0);
      if (p.pref.exprs)
        for (const Req& r : *p.pref.exprs) add_req(r);
    }
    R.pterm_off.push_back((int32_t)R.pt_weight.size());
    for (const std::string& n : u.place) R.place_name.push_back(S.id(n));
    R.place_off.push_back((int32_t)R.place_name.size());
    for (const auto& c : u.cur) {
      R.cur_name.push_back(S.id(c.first));
      R.cur_rep.push_back(c.second ? *c.second : 0);
      R.cur_has_rep.push_back(c.second ? 1 : 0);
    }
    R.cur_off.push_back((int32_t)R.cur_name.size());
    auto put = [&](const OMap<int64_t>& m, std::vector<int32_t>& off, std::vector<int32_t>& nm, std::vector<int64_t>& val) {
      for (const auto& kv : m) {
        nm.push_back(S.id(kv.first));
        val.push_back(kv.second);
      }
      off.push_back((int32_t)nm.size());
    };
    put(u.wt, R.wt_off, R.wt_name, R.wt_val);
    put(u.mn, R.min_off, R.min_name, R.min_val);
    put(u.mx, R.max_off, R.max_name, R.max_val);
    put(u.cap, R.cap_off, R.cap_name, R.cap_val);
    u = Unit();
  }
}

}  // namespace

// A caller's kad_strs, checked once on entry (as the packer's validate_columns does): n >= 0, offsets from 0 and
// never decreasing, data present when any string is non-empty — a decreasing offset would otherwise become a
// huge string length and an out-of-bounds read. A null `s` is valid where the argument is optional.
static bool strs_ok(const kad_strs* s) {
  if (!s) return true;
  if (s->n < 0) return false;
  if (s->n == 0) return !s->off || s->off[0] == 0;
  if (!s->off || s->off[0] != 0) return false;
  for (int32_t i = 0; i < s->n; ++i)
    if (s->off[i + 1] < s->off[i]) return false;
  return s->off[s->n] == 0 || s->bytes;
}

// policy_of[i]: -1 (no policy: the object is scheduled to no clusters) or an index into `policies`. Anything
// else is a caller bug (a stale or off-by-one index) that must not silently unschedule the object everywhere.
static bool policy_of_ok(const int32_t* policy_of, int n, int np) {
  if (!policy_of) return true;
  for (int i = 0; i < n; ++i)
    if (policy_of[i] < -1 || policy_of[i] >= np) return false;
  return true;
}

extern "C" int kad_units_from_objects(const kad_type_config* tc, const kad_strs* objects, const kad_strs* policies,
                                      const int32_t* policy_of, int threads, kad_units** out) {
  if (!tc || !objects || !out || !strs_ok(objects) || !strs_ok(policies) ||
      !policy_of_ok(policy_of, objects->n, policies ? policies->n : 0))
    return KAD_EINVAL;
  *out = nullptr;
  try {
    auto R = std::make_unique<kad_units>();
    const int n = objects->n;
    const int np = policies ? policies->n : 0;
    if (threads <= 0) threads = 1 << 20;
    auto text = [](const kad_strs* s, int i) {
      return sv(reinterpret_cast<const char*>(s->bytes) + s->off[i], (size_t)(s->off[i + 1] - s->off[i]));
    };
    std::vector<Policy> pols((size_t)np);
    parallel_for(np, threads, [&](int lo, int hi) {
      for (int i = lo; i < hi; ++i) load_policy(text(policies, i), pols[(size_t)i]);
    }, 64);
    std::unordered_map<std::string, int32_t> pol_index;
    for (int i = 0; i < np; ++i) pol_index[pols[(size_t)i].ns + '\0' + pols[(size_t)i].name] = i;  // the last wins
    Builder B{*tc, pols, pol_index, {"spec", "template"}, "/", !tc->replicas_spec || !*tc->replicas_spec};
    {
      const std::string path = tc->replicas_spec ? tc->replicas_spec : "";
      std::vector<std::string> parts;
      size_t a = 0;
      for (size_t i = 0; i <= path.size(); ++i)
        if (i == path.size() || path[i] == '.') {
          if (i > a) parts.push_back(path.substr(a, i - a));
          a = i + 1;
        }
      for (size_t i = 0; i < parts.size(); ++i) {
        B.replicas_fields.push_back(parts[i]);
        B.replicas_slash += (i ? "/" : "") + parts[i];
      }
    }
    std::vector<Unit> units((size_t)n);
    parallel_for(n, threads, [&](int lo, int hi) {
      JDoc d, ad;  // the object's nodes, an annotation's nodes (capacity kept across objects)
      for (int i = lo; i < hi; ++i) {
        Unit& u = units[(size_t)i];
        try {
          B.build(text(objects, i), u, d, ad, policy_of ? policy_of[i] : -2);
        } catch (const Fail& f) {
          const int32_t pol = u.policy;
          u = Unit();
          u.status = f.status;
          u.msg = f.msg;
          u.policy = pol;
        }
      }
    }, 256);
    R->status.assign((size_t)n, 0);
    R->unit_index.assign((size_t)n, -1);
    R->policy_index.assign((size_t)n, -1);
    R->msg.assign((size_t)n, std::string());
    merge(*R, *tc, units);
    *out = R.release();
    return KAD_OK;
  } catch (const std::bad_alloc&) {
    return KAD_ENOMEM;
  } catch (...) {
    return KAD_EINVAL;
  }
}

extern "C" int kad_units_view(const kad_units* u, kad_su_columns* c, const int32_t** status, const int32_t** unit_index,
                              const int32_t** policy_index) {
  if (!u) return KAD_EINVAL;
  if (status) *status = u->status.data();
  if (unit_index) *unit_index = u->unit_index.data();
  if (policy_index) *policy_index = u->policy_index.data();
  if (!c) return KAD_OK;
  std::memset(c, 0, sizeof *c);
  c->n_units = u->n_units;
  c->str.n = (int32_t)(u->st.off.size() - 1);
  c->str.off = u->st.off.data();
  c->str.bytes = u->st.bytes.data();
  c->group = u->group.data();
  c->version = u->version.data();
  c->kind = u->kind.data();
  c->namespace_ = u->ns.data();
  c->name = u->name.data();
  c->flags = u->flags.data();
  c->desired = u->desired.data();
  c->max_clusters = u->max_clusters.data();
  c->req_cpu = u->req_cpu.data();
  c->req_mem = u->req_mem.data();
  c->req_eph = u->req_eph.data();
  c->scalar_off = u->scalar_off.data();
  c->scalar_name = u->scalar_name.data();
  c->scalar_val = u->scalar_val.data();
  c->tol_off = u->tol_off.data();
  c->tol_key = u->tol_key.data();
  c->tol_op = u->tol_op.data();
  c->tol_value = u->tol_value.data();
  c->tol_effect = u->tol_effect.data();
  c->sel_off = u->sel_off.data();
  c->sel_key = u->sel_key.data();
  c->sel_value = u->sel_value.data();
  c->n_reqs = (int32_t)u->rq_key.size();
  c->rq_key = u->rq_key.data();
  c->rq_op = u->rq_op.data();
  c->rq_val_off = u->rq_val_off.data();
  c->rq_val = u->rq_val.data();
  c->rterm_off = u->rterm_off.data();
  c->rt_req = u->rt_req.data();
  c->rt_n_expr = u->rt_n_expr.data();
  c->rt_n_field = u->rt_n_field.data();
  c->pterm_off = u->pterm_off.data();
  c->pt_weight = u->pt_weight.data();
  c->pt_req = u->pt_req.data();
  c->pt_n_expr = u->pt_n_expr.data();
  c->place_off = u->place_off.data();
  c->place_name = u->place_name.data();
  c->cur_off = u->cur_off.data();
  c->cur_name = u->cur_name.data();
  c->cur_rep = u->cur_rep.data();
  c->cur_has_rep = u->cur_has_rep.data();
  c->wt_off = u->wt_off.data();
  c->wt_name = u->wt_name.data();
  c->wt_val = u->wt_val.data();
  c->min_off = u->min_off.data();
  c->min_name = u->min_name.data();
  c->min_val = u->min_val.data();
  c->max_off = u->max_off.data();
  c->max_name = u->max_name.data();
  c->max_val = u->max_val.data();
  c->cap_off = u->cap_off.data();
  c->cap_name = u->cap_name.data();
  c->cap_val = u->cap_val.data();
  return KAD_OK;
}

extern "C" const char* kad_units_message(const kad_units* u, int32_t i) {
  if (!u || i < 0 || (size_t)i >= u->msg.size()) return "";
  return u->msg[(size_t)i].c_str();
}

extern "C" void kad_units_free(kad_units* u) { delete u; }

struct kad_applied {
  std::vector<int32_t> status;
  std::vector<uint8_t> modified;  // applySchedulingResult's result
  std::vector<uint8_t> changed;   // the text changed (that, or the added trigger annotation)
  std::vector<int64_t> off{0};
  std::vector<uint8_t> bytes;
  std::vector<int64_t> doff{0};  // the written fields' new values, 3 per object
  std::vector<uint8_t> dbytes;
  std::vector<std::string> msg;
};

extern "C" int kad_apply_results(const kad_type_config* tc, const kad_strs* objects, const kad_strs* cluster_names,
                                 const int32_t* res_off, const int32_t* res_cluster, const int64_t* res_replicas,
                                 const uint8_t* follower, const int64_t* threshold_ns, const kad_strs* trigger,
                                 const uint8_t* ann_only, int threads, kad_applied** out) {
  if (!tc || !objects || !cluster_names || !res_off || !out || !strs_ok(objects) || !strs_ok(cluster_names) ||
      !strs_ok(trigger))
    return KAD_EINVAL;
  *out = nullptr;
  const int n = objects->n;
  if (trigger && trigger->n != n) return KAD_EINVAL;
  if (res_off[0] != 0) return KAD_EINVAL;
  if (n > 0 && res_off[n] > 0 && (!res_cluster || !res_replicas)) return KAD_EINVAL;
  for (int i = 0; i < n; ++i)
    if (res_off[i] < 0 || res_off[i + 1] < res_off[i]) return KAD_EINVAL;
  for (int32_t k = 0; n > 0 && k < res_off[n]; ++k)
    if (res_cluster[k] < 0 || res_cluster[k] >= cluster_names->n) return KAD_EINVAL;
  try {
    auto R = std::make_unique<kad_applied>();
    if (threads <= 0) threads = 1 << 20;
    auto text = [](const kad_strs* s, int i) {
      return sv(reinterpret_cast<const char*>(s->bytes) + s->off[i], (size_t)(s->off[i + 1] - s->off[i]));
    };
    Applier A{*tc, "/"};
    {
      const std::string path = tc->replicas_spec ? tc->replicas_spec : "";
      std::string slash;
      size_t a = 0;
      for (size_t i = 0; i <= path.size(); ++i)
        if (i == path.size() || path[i] == '.') {
          if (i > a) slash += (slash.empty() ? "" : "/") + path.substr(a, i - a);
          a = i + 1;
        }
      A.replicas_slash = "/" + slash;
    }
    R->status.assign((size_t)n, KAD_APPLY_OK);
    R->modified.assign((size_t)n, 0);
    R->changed.assign((size_t)n, 0);
    R->msg.assign((size_t)n, std::string());
    std::vector<std::string> texts((size_t)n);
    std::vector<std::string> deltas((size_t)n * Applier::N_DELTA);
    parallel_for(n, threads, [&](int lo, int hi) {
      JDoc d;
      for (int i = lo; i < hi; ++i) {
        const sv t = text(objects, i);
        try {
          uint32_t root;
          if (!parse(t, d, &root) || d.v[root].t != J_OBJ) fail(KAD_APPLY_BAD_JSON, "object: not a JSON object");
          std::vector<std::string> clusters;
          OMap<int64_t> desired;
          for (int32_t k = res_off[i]; k < res_off[i + 1]; ++k) {
            std::string name(text(cluster_names, res_cluster[k]));
            if (res_replicas[k] >= 0) desired.emplace_back(name, res_replicas[k]);
            clusters.push_back(std::move(name));
          }
          std::sort(clusters.begin(), clusters.end());
          clusters.erase(std::unique(clusters.begin(), clusters.end()), clusters.end());
          MV obj = mv_of(d, root, false);
          std::optional<int64_t> th;
          if (threshold_ns && threshold_ns[i] != INT64_MIN) th = threshold_ns[i];
          uint32_t wrote = 0;
          std::optional<sv> trig;
          if (trigger && trigger->off[i + 1] > trigger->off[i]) trig = text(trigger, i);
          bool trig_changed = false;
          const bool mod = A.apply(d, root, obj, wrote, clusters, desired, follower && follower[i], th, trig,
                                   ann_only && ann_only[i], trig_changed);
          R->modified[(size_t)i] = mod ? 1 : 0;
          R->changed[(size_t)i] = (mod || trig_changed) ? 1 : 0;
          if (mod || trig_changed) {
            emit(obj, texts[(size_t)i]);
            static const sv where[Applier::N_DELTA][2] = {{"spec", "placements"}, {"spec", "overrides"},
                                                          {"metadata", "annotations"}};
            for (int q = 0; q < Applier::N_DELTA; ++q)
              if (wrote & (1u << q)) emit(*obj.get(where[q][0])->get(where[q][1]), deltas[(size_t)i * Applier::N_DELTA + q]);
          }
        } catch (const Fail& f) {  // the object comes back as it was
          R->status[(size_t)i] = f.status;
          R->msg[(size_t)i] = f.msg;
          R->modified[(size_t)i] = 0;
          R->changed[(size_t)i] = 0;
          texts[(size_t)i].clear();
          for (int q = 0; q < Applier::N_DELTA; ++q) deltas[(size_t)i * Applier::N_DELTA + q].clear();
        }
      }
    }, 64);
    for (int i = 0; i < n; ++i) {
      if (R->changed[(size_t)i]) R->bytes.insert(R->bytes.end(), texts[(size_t)i].begin(), texts[(size_t)i].end());
      else {
        const sv t = text(objects, i);  // unchanged (or failed): the object as it was
        R->bytes.insert(R->bytes.end(), t.begin(), t.end());
      }
      R->off.push_back((int64_t)R->bytes.size());
      for (int q = 0; q < Applier::N_DELTA; ++q) {
        const std::string& x = deltas[(size_t)i * Applier::N_DELTA + q];
        R->dbytes.insert(R->dbytes.end(), x.begin(), x.end());
        R->doff.push_back((int64_t)R->dbytes.size());
      }
    }
    *out = R.release();
    return KAD_OK;
  } catch (const std::bad_alloc&) {
    return KAD_ENOMEM;
  } catch (...) {
    return KAD_EINVAL;
  }
}

extern "C" int kad_applied_view(const kad_applied* a, const int32_t** status, const uint8_t** modified,
                                const uint8_t** changed, kad_strs* texts) {
  if (!a) return KAD_EINVAL;
  if (status) *status = a->status.data();
  if (modified) *modified = a->modified.data();
  if (changed) *changed = a->changed.data();
  if (texts) {
    texts->n = (int32_t)a->status.size();
    texts->off = a->off.data();
    texts->bytes = a->bytes.data();
  }
  return KAD_OK;
}

extern "C" int kad_applied_fields(const kad_applied* a, kad_strs* fields) {
  if (!a || !fields) return KAD_EINVAL;
  fields->n = (int32_t)(a->doff.size() - 1);
  fields->off = a->doff.data();
  fields->bytes = a->dbytes.data();
  return KAD_OK;
}

extern "C" const char* kad_applied_message(const kad_applied* a, int32_t i) {
  if (!a || i < 0 || (size_t)i >= a->msg.size()) return "";
  return a->msg[(size_t)i].c_str();
}

extern "C" void kad_applied_free(kad_applied* a) { delete a; }

// ------------------------------------------------------------------ f4 host side: the trigger hash's object part
// computeSchedulingTriggerHash (schedulingtriggers.go:106-134) up to and including "clusterLabels": — the bytes
// objects.trigger_prefix builds — for a batch of object texts, with the policy lookup and the two annotation facts
// the reconcile needs next (the current hash annotation, the no-scheduling annotation).
struct kad_trigger_objs {
  std::vector<int32_t> status, policy_index;
  std::vector<uint8_t> flags;         // KAD_TRIG_HAS_HASH, KAD_TRIG_NO_SCHEDULING
  std::vector<int64_t> off{0}, hoff{0};
  std::vector<uint8_t> bytes, hbytes;  // prefixes; current hash annotation values
  std::vector<std::string> msg;
};

namespace {

constexpr sv KNOWN_SCHED_ANNS[] = {SCHEDULING_MODE_ANN, STICKY_ANN, TOLERATIONS_ANN, PLACEMENTS_ANN,
                                   SELECTOR_ANN, AFFINITY_ANN, MAX_CLUSTERS_ANN, FOLLOWS_OBJECT_ANN};

struct TrigOut {
  int status = KAD_OBJ_OK;
  int32_t policy = -1;
  uint8_t flags = 0;
  std::string prefix, hash, msg;
};

void trigger_one(const kad_type_config& tc, const std::vector<Policy>& pols,
                 const std::unordered_map<std::string, int32_t>& pol_index, const std::vector<std::string>& rfields,
                 bool replicas_empty, int32_t forced, sv text, JDoc& d, TrigOut& o) {
  uint32_t root;
  if (!parse(text, d, &root) || d.v[root].t != J_OBJ) fail(KAD_OBJ_BAD_JSON, "object: not a JSON object");
  const int64_t anns = Builder::string_map(d, root, "annotations");
  const int64_t labels = Builder::string_map(d, root, "labels");
  auto ann = [&](sv key) -> std::optional<sv> {
    if (anns < 0) return std::nullopt;
    const int64_t v = get(d, (uint32_t)anns, key);
    if (v < 0) return std::nullopt;
    return d.str((uint32_t)v);
  };
  // MatchedPolicyKey + lookup (scheduler.go:359-372), as Builder::build
  if (forced >= -1) {
    o.policy = forced >= 0 ? forced : -1;  // range-checked on entry (policy_of_ok)
  } else {
    std::optional<std::string> key;
    const int64_t pl = labels >= 0 ? get(d, (uint32_t)labels, POLICY_LABEL) : -1;
    const int64_t cl = labels >= 0 ? get(d, (uint32_t)labels, CLUSTER_POLICY_LABEL) : -1;
    if (pl >= 0 && tc.namespaced) {
      std::string ns;
      const int64_t meta = get(d, root, "metadata");
      const int64_t nsv = meta >= 0 && d.v[meta].t == J_OBJ ? get(d, (uint32_t)meta, "namespace") : -1;
      if (nsv >= 0 && d.v[nsv].t == J_STR) ns.assign(d.str((uint32_t)nsv));
      key = ns + '\0' + std::string(d.str((uint32_t)pl));
    } else if (cl >= 0) {
      key = std::string(1, '\0') + std::string(d.str((uint32_t)cl));
    }
    if (key) {
      auto it = pol_index.find(*key);
      if (it == pol_index.end()) {
        o.status = KAD_OBJ_POLICY_NOT_FOUND;
        return;
      }
      o.policy = it->second;
    }
  }
  const Policy* P = o.policy >= 0 ? &pols[(size_t)o.policy] : nullptr;
  if (P && !P->ok) fail(KAD_OBJ_POLICY_ERROR, P->err);
  // getReplicaCount (schedulingtriggers.go:171-186)
  int64_t replicas = 0;
  if (!replicas_empty) {
    uint32_t x = root;
    bool found = true;
    for (const std::string& f : rfields) {
      if (d.v[x].t != J_OBJ) fail(KAD_OBJ_UNIT_ERROR, "cannot access [spec template]: accessor error: not a map");
      const int64_t y = get(d, x, f);
      if (y < 0) {
        found = false;
        break;
      }
      x = (uint32_t)y;
    }
    if (found) {
      const JV& v = d.v[x];
      if (v.t != J_NUM || !v.isint || !v.fits) fail(KAD_OBJ_UNIT_ERROR, "cannot access [spec template]: expected int64");
      replicas = v.i;
    }
  }
  std::string& s = o.prefix;
  s += "{\"schedulingAnnotations\":[";
  {  // sortMap of the scheduling annotations: keys unique, bytewise order
    std::vector<std::pair<sv, sv>> kv;
    for (sv k : KNOWN_SCHED_ANNS)
      if (auto v = ann(k)) kv.emplace_back(k, *v);
    std::sort(kv.begin(), kv.end());
    for (size_t i = 0; i < kv.size(); ++i) {
      s += i ? ",{\"key\":" : "{\"key\":";
      emit_str(kv[i].first, s);
      s += ",\"value\":";
      emit_str(kv[i].second, s);
      s += '}';
    }
  }
  s += "],\"replicaCount\":" + std::to_string(replicas) +
       ",\"resourceRequest\":{\"millicpu\":0,\"memory\":0,\"ephemeralStorage\":0,\"scalarResources\":null}";
  if (P && P->spec.am) {
    if (auto v = ann(AUTO_MIGRATION_INFO_ANN)) {
      s += ",\"autoMigrationInfo\":";
      emit_str(*v, s);
    }
  }
  s += ",\"policyName\":";
  emit_str(P ? sv(P->name) : sv(), s);
  s += ",\"policyGeneration\":" + std::to_string(P ? P->generation : 0) + ",\"clusterLabels\":";
  if (auto h = ann(TRIGGER_HASH_ANN)) {
    o.flags |= KAD_TRIG_HAS_HASH;
    o.hash.assign(*h);
  }
  if (auto ns = ann(NO_SCHEDULING_ANN); ns && !ns->empty()) o.flags |= KAD_TRIG_NO_SCHEDULING;
  if (anns < 0) {
    const int64_t meta = get(d, root, "metadata");
    const int64_t an = meta >= 0 && d.v[meta].t == J_OBJ ? get(d, (uint32_t)meta, "annotations") : -1;
    if (an >= 0 && d.v[an].t != J_NULL) o.flags |= KAD_TRIG_ANN_NOT_MAP;
  }
}

}  // namespace

extern "C" int kad_trigger_prefixes(const kad_type_config* tc, const kad_strs* objects, const kad_strs* policies,
                                    const int32_t* policy_of, int threads, kad_trigger_objs** out) {
  if (!tc || !objects || !out || !strs_ok(objects) || !strs_ok(policies) ||
      !policy_of_ok(policy_of, objects->n, policies ? policies->n : 0))
    return KAD_EINVAL;
  *out = nullptr;
  try {
    auto R = std::make_unique<kad_trigger_objs>();
    const int n = objects->n, np = policies ? policies->n : 0;
    if (threads <= 0) threads = 1 << 20;
    auto text = [](const kad_strs* s, int i) {
      return sv(reinterpret_cast<const char*>(s->bytes) + s->off[i], (size_t)(s->off[i + 1] - s->off[i]));
    };
    std::vector<Policy> pols((size_t)np);
    parallel_for(np, threads, [&](int lo, int hi) {
      for (int i = lo; i < hi; ++i) load_policy(text(policies, i), pols[(size_t)i]);
    }, 64);
    std::unordered_map<std::string, int32_t> pol_index;
    for (int i = 0; i < np; ++i) pol_index[pols[(size_t)i].ns + '\0' + pols[(size_t)i].name] = i;
    std::vector<std::string> rfields{"spec", "template"};
    {
      const std::string path = tc->replicas_spec ? tc->replicas_spec : "";
      size_t a = 0;
      for (size_t i = 0; i <= path.size(); ++i)
        if (i == path.size() || path[i] == '.') {
          if (i > a) rfields.push_back(path.substr(a, i - a));
          a = i + 1;
        }
    }
    const bool replicas_empty = !tc->replicas_spec || !*tc->replicas_spec;
    std::vector<TrigOut> outs((size_t)n);
    parallel_for(n, threads, [&](int lo, int hi) {
      JDoc d;
      for (int i = lo; i < hi; ++i) {
        TrigOut& o = outs[(size_t)i];
        try {
          trigger_one(*tc, pols, pol_index, rfields, replicas_empty, policy_of ? policy_of[i] : -2, text(objects, i), d, o);
        } catch (const Fail& f) {
          const int32_t pol = o.policy;
          o = TrigOut();
          o.status = f.status;
          o.msg = f.msg;
          o.policy = pol;
        }
      }
    }, 256);
    R->status.resize((size_t)n);
    R->policy_index.resize((size_t)n);
    R->flags.resize((size_t)n);
    R->msg.resize((size_t)n);
    for (int i = 0; i < n; ++i) {
      TrigOut& o = outs[(size_t)i];
      R->status[(size_t)i] = o.status;
      R->policy_index[(size_t)i] = o.policy;
      R->flags[(size_t)i] = o.flags;
      R->msg[(size_t)i] = std::move(o.msg);
      R->bytes.insert(R->bytes.end(), o.prefix.begin(), o.prefix.end());
      R->off.push_back((int64_t)R->bytes.size());
      R->hbytes.insert(R->hbytes.end(), o.hash.begin(), o.hash.end());
      R->hoff.push_back((int64_t)R->hbytes.size());
    }
    *out = R.release();
    return KAD_OK;
  } catch (const std::bad_alloc&) {
    return KAD_ENOMEM;
  } catch (...) {
    return KAD_EINVAL;
  }
}

extern "C" int kad_trigger_objs_view(const kad_trigger_objs* t, const int32_t** status, const int32_t** policy_index,
                                     const uint8_t** flags, kad_strs* prefixes, kad_strs* current_hash) {
  if (!t) return KAD_EINVAL;
  if (status) *status = t->status.data();
  if (policy_index) *policy_index = t->policy_index.data();
  if (flags) *flags = t->flags.data();
  if (prefixes) *prefixes = kad_strs{(int32_t)t->status.size(), t->off.data(), t->bytes.data()};
  if (current_hash) *current_hash = kad_strs{(int32_t)t->status.size(), t->hoff.data(), t->hbytes.data()};
  return KAD_OK;
}

extern "C" const char* kad_trigger_objs_message(const kad_trigger_objs* t, int32_t i) {
  if (!t || i < 0 || (size_t)i >= t->msg.size()) return "";
  return t->msg[(size_t)i].c_str();
}

extern "C" void kad_trigger_objs_free(kad_trigger_objs* t) { delete t; }
