// Native batch packer (include/kad_pack.h): columnar SchedulingUnits → the
// kad_sched.h batch blob, byte-identical to kubeadmiral_amd/pack.py Batch.
//
// Passes (W units, R requirement-table entries, NT toleration sets):
//   1. per requirement entry, in parallel: labels.NewRequirement validation
//      (apimachinery v0.26.6 labels/selector.go) and the requirement words of
//      both uses (label expression, metadata.name field selector);
//   2. serial, in unit order: interning — requirement words → batch-wide ids
//      and toleration lists → toleration-set ids, in exactly the order pack.py
//      assigns them (first use), so the blob is byte-identical;
//   3. per unit, in parallel: flags, fixed columns and the length of every
//      CSR row; serial prefix sums lay out the blob;
//   4. per unit, in parallel: the CSR rows written in place (programs,
//      placement / current / preference lists sorted by snapshot id, Key()
//      bytes); per toleration set: tolerated-taint masks
//      (Toleration.ToleratesTaint, k8s.io/api v0.26.6).
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/kad_pack.h"
#include "kad_pool.h"

namespace {

using sv = std::string_view;

constexpr int ALIGN = 256;
constexpr int OP_IN = 1, OP_NOTIN = 2, OP_EXISTS = 3, OP_DNE = 4, OP_GT = 5, OP_LT = 6, OP_EQ = 7, OP_TRUE = 8,
              OP_FALSE = 9, OP_NAME_EQ = 10, OP_NAME_NE = 11;

struct Strs {
  const int64_t* off = nullptr;
  const uint8_t* bytes = nullptr;
  int32_t n = 0;
  sv operator[](int i) const {
    return sv(reinterpret_cast<const char*>(bytes) + off[i], (size_t)(off[i + 1] - off[i]));
  }
};
Strs strs(const kad_strs& s) { return Strs{s.off, s.bytes, s.n}; }

// ------------------------------------------------ apimachinery / k8s.io/api
bool dns1123_subdomain(sv s) {  // [a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*
  if (s.empty()) return false;
  size_t i = 0;
  while (true) {
    size_t j = i;
    while (j < s.size() && s[j] != '.') j++;
    if (j == i) return false;
    auto alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!alnum(s[i]) || !alnum(s[j - 1])) return false;
    for (size_t k = i; k < j; k++)
      if (!alnum(s[k]) && s[k] != '-') return false;
    if (j == s.size()) return true;
    i = j + 1;
  }
}
bool alnum_any(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
bool qname_part(sv s) {  // ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9], 1..63
  if (s.empty() || s.size() > 63) return false;
  if (!alnum_any(s.front()) || !alnum_any(s.back())) return false;
  for (char c : s)
    if (!alnum_any(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}
bool is_qualified_name(sv v) {  // validation.IsQualifiedName
  const size_t a = v.find('/');
  if (a == sv::npos) return qname_part(v);
  if (v.find('/', a + 1) != sv::npos) return false;
  const sv prefix = v.substr(0, a), name = v.substr(a + 1);
  if (prefix.empty() || prefix.size() > 253 || !dns1123_subdomain(prefix)) return false;
  return qname_part(name);
}
bool is_valid_label_value(sv v) {  // validation.IsValidLabelValue (empty allowed)
  return v.empty() || qname_part(v);
}
bool parse_int64(sv s, int64_t* out) {  // strconv.ParseInt(s, 10, 64)
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i == s.size()) return false;
  uint64_t v = 0;
  const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  for (; i < s.size(); i++) {
    const char c = s[i];
    if (c < '0' || c > '9') return false;
    const uint64_t d = (uint64_t)(c - '0');
    if (v > (lim - d) / 10) return false;
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}
int label_op(sv op) {
  if (op == "In") return OP_IN;
  if (op == "NotIn") return OP_NOTIN;
  if (op == "Exists") return OP_EXISTS;
  if (op == "DoesNotExist") return OP_DNE;
  if (op == "Gt") return OP_GT;
  if (op == "Lt") return OP_LT;
  return 0;
}

// f(a, b) over [0, n) split into contiguous ranges on up to `threads` threads; `grain` = the fewest
// items worth a thread of their own
template <class F>
void parallel_for(int n, int threads, F f, int grain = 1024) {
  if (n <= 0) return;
  if (threads <= 1 || n < 2 * grain) {
    f(0, n);
    return;
  }
  const int T = std::min(threads, (n + grain - 1) / grain);
  // the library's persistent workers (kad_pool.h): T ranges, run by at most pool().threads() at a time
  kadpool::pool().run(T, [&](int t) { f((int)((int64_t)n * t / T), (int)((int64_t)n * (t + 1) / T)); });
}

struct WordsHash {
  size_t operator()(const std::vector<int32_t>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int32_t x : v) h = (h ^ (uint32_t)x) * 1099511628211ull;
    return (size_t)h;
  }
};

size_t align_up(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }
struct IdSet;
const std::vector<int32_t>& sorted_unique(const std::vector<int32_t>& cs, int i0, int i1, IdSet& set,
                                          std::vector<int32_t>& out);

// A per-thread set of snapshot cluster ids in [0, C): a bitmap whose touched words are scanned in order,
// so sort + unique of a unit's few dozen ids costs one pass plus (max - min) / 64 words. Used when that
// range is short next to the list (else the caller sorts).
struct IdSet {
  std::vector<uint64_t> bm;
  int lo = INT32_MAX, hi = -1;
  explicit IdSet(int C) : bm(((size_t)(C > 0 ? C : 1) + 63) / 64, 0ull) {}
  static bool worth(int lo_id, int hi_id, size_t n) { return hi_id < lo_id || (size_t)((hi_id >> 6) - (lo_id >> 6)) <= 2 * n + 8; }
  void add(int c) {
    bm[(size_t)c >> 6] |= 1ull << (c & 63);
    lo = c < lo ? c : lo;
    hi = c > hi ? c : hi;
  }
  // f(id) for every member in ascending order; the set is empty afterwards
  template <class F>
  void drain(F f) {
    if (hi >= 0)
      for (int wd = lo >> 6; wd <= (hi >> 6); wd++) {
        uint64_t x = bm[wd];
        bm[wd] = 0;
        while (x) {
          f(wd * 64 + __builtin_ctzll(x));
          x &= x - 1;
        }
      }
    lo = INT32_MAX;
    hi = -1;
  }
  // the sorted distinct ids >= 0 among cs[i0, i1) into out
  static void sorted_unique_into(const std::vector<int32_t>& cs, int i0, int i1, IdSet& set, std::vector<int32_t>& out) {
    out.clear();
    int lo_id = INT32_MAX, hi_id = -1;
    size_t nn = 0;
    for (int i = i0; i < i1; i++)
      if (cs[i] >= 0) {
        lo_id = std::min(lo_id, cs[i]);
        hi_id = std::max(hi_id, cs[i]);
        nn++;
      }
    if (worth(lo_id, hi_id, nn)) {
      for (int i = i0; i < i1; i++)
        if (cs[i] >= 0) set.add(cs[i]);
      set.drain([&](int c) { out.push_back(c); });
      return;
    }
    for (int i = i0; i < i1; i++)
      if (cs[i] >= 0) out.push_back(cs[i]);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
  }
  int count_and_clear() {
    int n = 0;
    if (hi >= 0)
      for (int wd = lo >> 6; wd <= (hi >> 6); wd++) {
        n += __builtin_popcountll(bm[wd]);
        bm[wd] = 0;
      }
    lo = INT32_MAX;
    hi = -1;
    return n;
  }
};
const std::vector<int32_t>& sorted_unique(const std::vector<int32_t>& cs, int i0, int i1, IdSet& set,
                                          std::vector<int32_t>& out) {
  IdSet::sorted_unique_into(cs, i0, i1, set, out);
  return out;
}

// Open-addressing index of (hash, id) slots: no allocation per entry, reset by one fill and kept across
// packs. On a hash match the caller's predicate compares contents, so distinct keys with equal hashes
// coexist (each content is inserted once; a probe finds only its equal).
struct FlatIndex {
  std::vector<uint64_t> hs;
  std::vector<int32_t> ids;
  size_t mask = 0, n = 0;
  static uint64_t mix(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return h;
  }
  void reset(size_t expect = 32) {
    size_t cap = 64;
    while (cap < 2 * expect) cap <<= 1;
    if (ids.size() < cap) {
      hs.assign(cap, 0);
      ids.assign(cap, -1);
    } else {
      std::fill(ids.begin(), ids.end(), -1);
    }
    mask = ids.size() - 1;
    n = 0;
  }
  // the id of the entry equal to the probe (same(id) on a hash match), else adds make_id()'s
  template <class Same, class Make>
  int32_t find_or_add(uint64_t h, Same same, Make make_id) {
    if (2 * (n + 1) > ids.size()) grow();
    size_t i = mix(h) & mask;
    for (; ids[i] >= 0; i = (i + 1) & mask)
      if (hs[i] == h && same(ids[i])) return ids[i];
    const int32_t id = make_id();
    hs[i] = h;
    ids[i] = id;
    n++;
    return id;
  }
  void grow() {
    std::vector<uint64_t> oh;
    std::vector<int32_t> oi;
    oh.swap(hs);
    oi.swap(ids);
    const size_t cap = std::max<size_t>(64, 2 * oi.size());
    hs.assign(cap, 0);
    ids.assign(cap, -1);
    mask = cap - 1;
    for (size_t j = 0; j < oi.size(); j++)
      if (oi[j] >= 0) {
        size_t i = mix(oh[j]) & mask;
        while (ids[i] >= 0) i = (i + 1) & mask;
        hs[i] = oh[j];
        ids[i] = oi[j];
      }
  }
};

// one chunk of units' interning state (kad_pack_batch step 2), kept across packs
struct InternChunk {
  FlatIndex req_ix;
  std::vector<sv> reqs;                            // local id → words
  std::deque<std::array<int32_t, 3>> extra_words;  // selector Equals words (stable addresses)
  FlatIndex eq_ix;
  std::vector<int64_t> eq_code;                    // selector entry → its (key, value) code
  std::vector<int32_t> eq_req;                     //   and its local requirement id
  FlatIndex tol_ix;
  std::vector<int> tol_rows;                       // local set → its first unit
  void reset() {
    req_ix.reset();
    reqs.clear();
    extra_words.clear();
    eq_ix.reset();
    eq_code.clear();
    eq_req.clear();
    tol_ix.reset();
    tol_rows.clear();
  }
};

}  // namespace

struct kad_packer {
  using Map = std::unordered_map<sv, int>;
  std::string err;
  int C = 0, TW = 1;
  uint64_t fingerprint = 0;
  // vocabulary strings are owned here (a deque never moves its elements: the views stay valid)
  std::deque<std::string> own;
  Map name_id, scalar_id, label_key_id, gvk_id;
  std::vector<Map> label_vals;
  std::vector<std::string> taint_key, taint_value, taint_effect;
  // the last packed blob (kad_packer_take / kad_packer_blob): page-locked host memory (one DMA to the GPU),
  // kept across packs (grown when needed, so repeated packs touch no new pages)
  uint8_t* out = nullptr;
  size_t out_n = 0, out_cap = 0;
  bool out_pinned = false;
  int take_threads = 1;
  // per-pack scratch arrays, kept across packs: resizing a kept vector to the same size touches no new
  // pages and initialises nothing (every array below is fully written, or explicitly filled, per pack)
  struct Scratch {
    std::vector<uint8_t> valid, fvalid, is_field;
    std::vector<int64_t> eoff, sel_code, maxc, desired, out_len, o_out;
    std::vector<int32_t> wbuf, elen, fw, egid, fgid, sgid, tolset, owner, unit_chunk, gvk, n_sreq, n_fp, n_sp,
        n_place, n_cur, n_pref, n_key, nr, o_sreq, o_fp, o_sp, o_place, o_cur, o_pref, o_key, req_off;
    std::vector<uint64_t> tol_hash, fo_hash;
    std::vector<uint32_t> flags;
    std::vector<int32_t> fo_canon, req_gid, tol_gid, flat_chunk;
    // per string id of the batch's string table, filled lazily by the threads that meet it (every writer
    // stores the same value): 0 unknown, 1 yes, 2 no / label key id + 2 (0 unknown)
    std::vector<uint8_t> m_qname, m_lvalue, m_op;
    std::vector<int32_t> m_kid, m_cid;  // m_cid: cluster-name string → snapshot id + 2 (0 unknown)
    // map / set entries' snapshot ids (kept: ~90 entries per C4 unit, 350 MB of fresh pages per 1M-unit pack)
    std::vector<int32_t> place_c, cur_c, wt_c, min_c, max_c, cap_c;
    std::vector<InternChunk> chunks;
  } sc;

  uint8_t* reserve(size_t n) {
    if (n <= out_cap && out) return out;
    release();
    void* p = nullptr;
    if (hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess && p) {
      out_pinned = true;
    } else {  // no HIP device here (CPU-only hosts, tests): ordinary memory
      (void)hipGetLastError();
      p = std::malloc(n);
      out_pinned = false;
    }
    out = static_cast<uint8_t*>(p);
    out_cap = out ? n : 0;
    return out;
  }
  void release() {
    if (out) {
      if (out_pinned)
        (void)hipHostFree(out);
      else
        std::free(out);
    }
    out = nullptr;
    out_cap = 0;
  }
  ~kad_packer() { release(); }

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  sv keep(std::string s) {
    own.push_back(std::move(s));
    return sv(own.back());
  }
  static void gvk_key(std::string& s, sv g, sv v, sv k) {
    s.clear();
    s.append(g).push_back('\0');
    s.append(v).push_back('\0');
    s.append(k);
  }
  static int find(const Map& m, sv s) {
    auto it = m.find(s);
    return it == m.end() ? -1 : it->second;
  }

  // label_req / eq_req / field_req of pack.py _Compiler
  void label_words(sv key, int op, const int32_t* vals, int nv, const Strs& S, std::vector<int32_t>& w) const {
    w.clear();
    const int kid = find(label_key_id, key);
    if (kid < 0) {
      w = {(op == OP_NOTIN || op == OP_DNE) ? OP_TRUE : OP_FALSE, -1};
      return;
    }
    if (op == OP_IN || op == OP_NOTIN) {
      const auto& vocab = label_vals[kid];
      w.push_back(0);
      w.push_back(kid);
      for (int i = 0; i < nv; i++) {
        auto it = vocab.find(S[vals[i]]);
        if (it != vocab.end()) w.push_back(it->second);
      }
      std::sort(w.begin() + 2, w.end());
      w.erase(std::unique(w.begin() + 2, w.end()), w.end());
      if (w.size() == 2) {
        w = {op == OP_IN ? OP_FALSE : OP_TRUE, -1};
        return;
      }
      w[0] = op | ((int32_t)(w.size() - 2) << 8);
      return;
    }
    if (op == OP_EXISTS || op == OP_DNE) {
      w = {op, kid};
      return;
    }
    int64_t thr = 0;
    parse_int64(S[vals[0]], &thr);
    const uint64_t u = (uint64_t)thr;
    w = {op | (2 << 8), kid, (int32_t)(uint32_t)(u & 0xFFFFFFFFu), (int32_t)(uint32_t)(u >> 32)};
  }
  void eq_words(sv key, sv value, std::vector<int32_t>& w) const {
    const int kid = find(label_key_id, key);
    if (kid < 0) {
      w = {OP_FALSE, -1};
      return;
    }
    auto it = label_vals[kid].find(value);
    if (it == label_vals[kid].end()) {
      w = {OP_FALSE, -1};
      return;
    }
    w = {OP_EQ | (1 << 8), kid, it->second};
  }
  void field_words(sv key, sv op, sv v, std::vector<int32_t>& w) const {
    const bool eq = op == "In";
    if (key == "metadata.name") {
      w = {eq ? OP_NAME_EQ : OP_NAME_NE, find(name_id, v)};
      return;
    }
    const bool hit = v.empty();  // fields.Set.Get of a missing key reads as ""
    w = {hit == eq ? OP_TRUE : OP_FALSE, -1};
  }
};

// The columns come from another language's shim: every offset array must be monotone from 0, every
// string id and requirement range in bounds, before any pass indexes with them.
static int validate_columns(kad_packer* P, const kad_su_columns* su, int threads) {
  const int W = su->n_units, NS = su->str.n, R = su->n_reqs;
  if (NS < 0 || R < 0 || !su->str.off) return P->fail(KAD_EINVAL, "bad string table / requirement count");
  if (su->str.off[0] != 0) return P->fail(KAD_EINVAL, "string offsets must start at 0");
  // monotone offsets, checked in parallel pieces (each piece also checks its first step from the previous one)
  auto monotone = [&](const auto* off, int n) -> bool {
    std::atomic<bool> ok{true};
    parallel_for(n, threads, [&](int lo, int hi) {
      bool good = true;
      for (int i = lo; i < hi; i++) good &= off[i + 1] >= off[i];
      if (!good) ok = false;
    }, 1 << 15);
    return ok;
  };
  if (!monotone(su->str.off, NS)) return P->fail(KAD_EINVAL, "string offsets must be non-decreasing");
  std::atomic<bool> bad{false};
  auto ids_ok = [&](const int32_t* a, int64_t n) {
    parallel_for((int)n, threads, [&](int lo, int hi) {
      for (int i = lo; i < hi; i++)
        if (a[i] < 0 || a[i] >= NS) bad = true;
    });
  };
  auto csr = [&](const int32_t* off, int n, int64_t* total) -> bool {
    if (!off || off[0] != 0) return false;
    if (!monotone(off, n)) return false;
    *total = off[n];
    return true;
  };
  ids_ok(su->group, W);
  ids_ok(su->version, W);
  ids_ok(su->kind, W);
  ids_ok(su->namespace_, W);
  ids_ok(su->name, W);
  int64_t n;
  struct G {
    const int32_t* off;
    std::vector<const int32_t*> ids;
  };
  const G groups[] = {{su->scalar_off, {su->scalar_name}}, {su->tol_off, {su->tol_key, su->tol_op, su->tol_value, su->tol_effect}},
                      {su->sel_off, {su->sel_key, su->sel_value}}, {su->place_off, {su->place_name}},
                      {su->cur_off, {su->cur_name}}, {su->wt_off, {su->wt_name}}, {su->min_off, {su->min_name}},
                      {su->max_off, {su->max_name}}, {su->cap_off, {su->cap_name}}};
  for (const G& g : groups) {
    if (!csr(g.off, W, &n)) return P->fail(KAD_EINVAL, "a per-unit CSR offset array is not monotone from 0");
    for (const int32_t* a : g.ids) ids_ok(a, n);
  }
  int64_t nrt, npt, nv;
  if (!csr(su->rterm_off, W, &nrt) || !csr(su->pterm_off, W, &npt) || !csr(su->rq_val_off, R, &nv))
    return P->fail(KAD_EINVAL, "term / requirement offsets are not monotone from 0");
  ids_ok(su->rq_key, R);
  ids_ok(su->rq_op, R);
  ids_ok(su->rq_val, nv);
  std::atomic<bool> tbad{false};
  parallel_for((int)nrt, threads, [&](int lo, int hi) {
    for (int t = lo; t < hi; t++)
      if (su->rt_req[t] < 0 || su->rt_n_expr[t] < 0 || su->rt_n_field[t] < 0 ||
          (int64_t)su->rt_req[t] + su->rt_n_expr[t] + su->rt_n_field[t] > R)
        tbad = true;
  }, 1 << 15);
  if (tbad) return P->fail(KAD_EINVAL, "required term outside the requirement table");
  parallel_for((int)npt, threads, [&](int lo, int hi) {
    for (int t = lo; t < hi; t++)
      if (su->pt_req[t] < 0 || su->pt_n_expr[t] < 0 || (int64_t)su->pt_req[t] + su->pt_n_expr[t] > R) tbad = true;
  }, 1 << 15);
  if (tbad) return P->fail(KAD_EINVAL, "preferred term outside the requirement table");
  if (bad) return P->fail(KAD_EINVAL, "string id out of range");
  return 0;
}

extern "C" {

// kad_packer_create's message for kad_packer_error(NULL) (no packer exists to carry it)
static thread_local std::string g_create_err;

// one vocabulary string array: n >= 0, offsets from 0, non-decreasing, bytes present when non-empty
static bool strs_ok(const kad_strs& s) {
  if (s.n < 0) return false;
  if (s.n == 0) return true;
  if (!s.off || s.off[0] != 0) return false;
  for (int i = 0; i < s.n; i++)
    if (s.off[i + 1] < s.off[i]) return false;
  return s.off[s.n] == 0 || s.bytes;
}

// the vocabulary a caller hands over (cgo / ctypes) is checked as carefully as the unit columns:
// every array well formed, the GVK and taint triples of equal length, label value ranges in bounds
static const char* check_vocab(const kad_pack_vocab* v) {
  const kad_strs* all[] = {&v->cluster_names, &v->scalar_names, &v->gvk_group, &v->gvk_version, &v->gvk_kind,
                           &v->label_keys, &v->label_vals, &v->taint_key, &v->taint_value, &v->taint_effect};
  for (const kad_strs* s : all)
    if (!strs_ok(*s)) return "a vocabulary string array has bad offsets (n < 0, not from 0, decreasing, or no bytes)";
  if (v->gvk_version.n != v->gvk_group.n || v->gvk_kind.n != v->gvk_group.n)
    return "gvk_group, gvk_version and gvk_kind must have the same length";
  if (v->taint_value.n != v->taint_key.n || v->taint_effect.n != v->taint_key.n)
    return "taint_key, taint_value and taint_effect must have the same length";
  const int K = v->label_keys.n;
  if (K > 0 || v->label_val_off) {
    if (!v->label_val_off) return "label_val_off is null";
    if (v->label_val_off[0] != 0) return "label_val_off[0] must be 0";
    for (int k = 0; k < K; k++)
      if (v->label_val_off[k + 1] < v->label_val_off[k]) return "label_val_off must be non-decreasing";
    if (v->label_val_off[K] > v->label_vals.n) return "label_val_off[n_keys] exceeds label_vals.n";
  }
  if (v->n_taint_words < 1 || (int64_t)v->n_taint_words * 64 < v->taint_key.n)
    return "n_taint_words must be >= 1 and cover every taint id";
  return nullptr;
}

static int packer_create_impl(const kad_pack_vocab* v, kad_packer** out) {
  if (!v || !out) {
    g_create_err = "null vocabulary or output pointer";
    return KAD_EINVAL;
  }
  if (const char* e = check_vocab(v)) {
    g_create_err = e;
    return KAD_EINVAL;
  }
  g_create_err.clear();
  auto* p = new kad_packer();
  const Strs names = strs(v->cluster_names), sc = strs(v->scalar_names), gg = strs(v->gvk_group),
             gv = strs(v->gvk_version), gk = strs(v->gvk_kind), lk = strs(v->label_keys), lv = strs(v->label_vals),
             tk = strs(v->taint_key), tv = strs(v->taint_value), te = strs(v->taint_effect);
  p->C = names.n;
  p->TW = v->n_taint_words;
  p->fingerprint = v->fingerprint;
  for (int i = 0; i < names.n; i++) p->name_id.emplace(p->keep(std::string(names[i])), i);
  for (int i = 0; i < sc.n; i++) p->scalar_id.emplace(p->keep(std::string(sc[i])), i);
  std::string key;
  for (int i = 0; i < gg.n; i++) {
    kad_packer::gvk_key(key, gg[i], gv[i], gk[i]);
    p->gvk_id.emplace(p->keep(key), i);
  }
  p->label_vals.resize(lk.n);
  for (int k = 0; k < lk.n; k++) {
    p->label_key_id.emplace(p->keep(std::string(lk[k])), k);
    for (int j = v->label_val_off[k]; j < v->label_val_off[k + 1]; j++)
      p->label_vals[k].emplace(p->keep(std::string(lv[j])), j - v->label_val_off[k]);
  }
  for (int i = 0; i < tk.n; i++) {
    p->taint_key.emplace_back(tk[i]);
    p->taint_value.emplace_back(tv[i]);
    p->taint_effect.emplace_back(te[i]);
  }
  *out = p;
  return KAD_OK;
}

int kad_packer_destroy(kad_packer* p) {
  delete p;
  return KAD_OK;
}

const char* kad_packer_error(kad_packer* p) { return p ? p->err.c_str() : g_create_err.c_str(); }

static int packer_take_impl(kad_packer* p, void* dst, size_t cap) {
  if (!p || (!dst && p->out_n)) return KAD_EINVAL;
  if (cap < p->out_n) return p->fail(KAD_EINVAL, "destination smaller than the packed blob");
  const size_t n = p->out_n, chunk = 4u << 20;
  const int pieces = (int)((n + chunk - 1) / chunk);
  parallel_for(pieces, p->take_threads, [&](int a, int b) {
    for (int i = a; i < b; i++) {
      const size_t o = (size_t)i * chunk;
      std::memcpy(static_cast<uint8_t*>(dst) + o, p->out + o, std::min(chunk, n - o));
    }
  }, 1);
  p->out_n = 0;
  return KAD_OK;
}

int kad_packer_blob(kad_packer* p, const void** data, size_t* nbytes) {
  if (!p || !data || !nbytes) return KAD_EINVAL;
  if (!p->out_n) return p->fail(KAD_ESTATE, "no packed blob");
  *data = p->out;
  *nbytes = p->out_n;
  return KAD_OK;
}

static int pack_batch_impl(kad_packer* P, const kad_profile* prof, const kad_su_columns* su, int threads,
                           size_t* nbytes, kad_pack_stats* stats) {
  if (!P || !prof || !su || !nbytes) return KAD_EINVAL;
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  P->take_threads = threads;
  const int W = su->n_units;
  if (W < 0) return P->fail(KAD_EINVAL, "n_units < 0");
  const Strs S{su->str.off, su->str.bytes, su->str.n};
  const int C = P->C, TW = P->TW;
#if defined(KAD_PHASE_PROF) || defined(KAD_TUNING)
  static const bool tm = getenv("KAD_PACK_TIMING") != nullptr;  // measurement builds only
#else
  constexpr bool tm = false;
#endif
  auto t_prev = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[kad_pack] %-10s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t_prev).count());
    t_prev = t;
  };
  if (int r = validate_columns(P, su, threads)) return r;
  lap("validate");
  const bool select_max = prof->select_plugin == KAD_PL_MAX_CLUSTER;
  const bool place_on = prof->filter_mask & (1u << KAD_PL_PLACEMENT_FILTER);
  const int R = su->n_reqs;

  // ---- 1. requirement entries (parallel): validity, expression words into one flat buffer (a slot of
  // 2 + max(nv, 2) words per entry), field words only for entries a required term uses as a field
  auto& X = P->sc;
  // fill in parallel (kept scratch: no fresh pages)
  auto pfill = [&](auto& v, auto x) {
    parallel_for((int)std::min<size_t>(v.size(), INT32_MAX), threads, [&](int a, int b) {
      std::fill(v.begin() + a, v.begin() + b, x);
    }, 1 << 16);
  };
  auto& valid = X.valid;
  auto& fvalid = X.fvalid;
  auto& is_field = X.is_field;
  auto& eoff = X.eoff;
  valid.resize(R);
  fvalid.resize(R);
  is_field.resize(R);
  pfill(is_field, (uint8_t)0);
  eoff.resize((size_t)R + 1);
  eoff[0] = 0;
  for (int r = 0; r < R; r++) eoff[r + 1] = eoff[r] + 2 + std::max(2, su->rq_val_off[r + 1] - su->rq_val_off[r]);
  auto& wbuf = X.wbuf;
  auto& elen = X.elen;
  auto& fw = X.fw;
  wbuf.resize((size_t)eoff[R]);
  elen.resize(R);
  fw.resize(2 * (size_t)R);
  lap("eoff");
  {
    const int nterms = W ? su->rterm_off[W] : 0;
    parallel_for(nterms, threads, [&](int a, int b) {
      for (int t = a; t < b; t++) {
        const int g0 = su->rt_req[t] + su->rt_n_expr[t];
        for (int e = g0; e < g0 + su->rt_n_field[t]; e++) is_field[e] = 1;
      }
    });
  }
  // string facts memoised per string id (keys, ops and values repeat across requirements)
  const int NSTR = su->str.n;
  X.m_qname.resize(NSTR);
  X.m_lvalue.resize(NSTR);
  X.m_op.resize(NSTR);
  X.m_kid.resize(NSTR);
  X.m_cid.resize(NSTR);
  pfill(X.m_cid, (int32_t)0);
  pfill(X.m_qname, (uint8_t)0);
  pfill(X.m_lvalue, (uint8_t)0);
  pfill(X.m_op, (uint8_t)0);
  pfill(X.m_kid, (int32_t)0);
  auto memo8 = [](uint8_t* slot, auto compute) -> uint8_t {
    uint8_t f = __atomic_load_n(slot, __ATOMIC_RELAXED);
    if (!f) {
      f = compute();
      __atomic_store_n(slot, f, __ATOMIC_RELAXED);
    }
    return f;
  };
  auto qname_ok = [&](int32_t id) {
    return memo8(&X.m_qname[id], [&] { return (uint8_t)(is_qualified_name(S[id]) ? 1 : 2); }) == 1;
  };
  auto lvalue_ok = [&](int32_t id) {
    return memo8(&X.m_lvalue[id], [&] { return (uint8_t)(is_valid_label_value(S[id]) ? 1 : 2); }) == 1;
  };
  auto op_of = [&](int32_t id) { return (int)memo8(&X.m_op[id], [&] { return (uint8_t)(label_op(S[id]) + 1); }) - 1; };
  auto kid_of = [&](int32_t id) {
    int32_t k = __atomic_load_n(&X.m_kid[id], __ATOMIC_RELAXED);
    if (!k) {
      k = kad_packer::find(P->label_key_id, S[id]) + 2;
      __atomic_store_n(&X.m_kid[id], k, __ATOMIC_RELAXED);
    }
    return k - 2;
  };
  parallel_for(R, threads, [&](int a, int b) {
    std::vector<int32_t> tmp;
    // (key id, value string) → value id, a direct-mapped cache per thread (one value string may belong to
    // several keys' vocabularies: a shared per-string slot would bounce between threads)
    constexpr int VC = 1 << 14;
    std::vector<int64_t> vc_key(VC, -1);
    std::vector<int32_t> vc_val(VC);
    auto vid_of = [&](int kid, int32_t id) {  // the value's id in key kid's vocabulary (-1: absent)
      const int64_t k = ((int64_t)kid << 32) | (uint32_t)id;
      const size_t slot = (size_t)(FlatIndex::mix((uint64_t)k) & (VC - 1));
      if (vc_key[slot] == k) return vc_val[slot];
      const int32_t v = kad_packer::find(P->label_vals[kid], S[id]);
      vc_key[slot] = k;
      vc_val[slot] = v;
      return v;
    };
    for (int r = a; r < b; r++) {
      const int32_t key_id = su->rq_key[r];
      const int v0 = su->rq_val_off[r], nv = su->rq_val_off[r + 1] - v0;
      const int32_t* vals = su->rq_val + v0;
      const int op = op_of(su->rq_op[r]);
      bool ok = op != 0 && qname_ok(key_id);
      if (ok && (op == OP_IN || op == OP_NOTIN)) ok = nv > 0;
      if (ok && (op == OP_EXISTS || op == OP_DNE)) ok = nv == 0;
      if (ok && (op == OP_GT || op == OP_LT)) {
        int64_t x;
        ok = nv == 1 && parse_int64(S[vals[0]], &x);
      }
      for (int i = 0; ok && i < nv; i++) ok = lvalue_ok(vals[i]);
      valid[r] = ok;
      elen[r] = 0;
      if (ok) {
        // label_words on memoised ids (same words)
        const int kid = kid_of(key_id);
        tmp.clear();
        if (kid < 0) {
          tmp = {(op == OP_NOTIN || op == OP_DNE) ? OP_TRUE : OP_FALSE, -1};
        } else if (op == OP_IN || op == OP_NOTIN) {
          tmp.push_back(0);
          tmp.push_back(kid);
          for (int i = 0; i < nv; i++) {
            const int32_t v = vid_of(kid, vals[i]);
            if (v >= 0) tmp.push_back(v);
          }
          std::sort(tmp.begin() + 2, tmp.end());
          tmp.erase(std::unique(tmp.begin() + 2, tmp.end()), tmp.end());
          if (tmp.size() == 2)
            tmp = {op == OP_IN ? OP_FALSE : OP_TRUE, -1};
          else
            tmp[0] = op | ((int32_t)(tmp.size() - 2) << 8);
        } else {
          P->label_words(S[key_id], op, vals, nv, S, tmp);
        }
        std::memcpy(wbuf.data() + eoff[r], tmp.data(), 4 * tmp.size());
        elen[r] = (int32_t)tmp.size();
      }
      fvalid[r] = (op == OP_IN || op == OP_NOTIN) && nv == 1;
      if (fvalid[r] && is_field[r]) {
        P->field_words(S[key_id], S[su->rq_op[r]], S[vals[0]], tmp);
        fw[2 * (size_t)r] = tmp[0];
        fw[2 * (size_t)r + 1] = tmp[1];
      }
    }
  });
  lap("reqwords");
  // ClusterSelector entries (parallel): SelectorFromSet's Equals as (key id, value id), -1 = absent
  const int64_t n_sel_total = W ? su->sel_off[W] : 0;
  auto& sel_code = X.sel_code;
  sel_code.resize((size_t)n_sel_total);
  parallel_for((int)n_sel_total, threads, [&](int a, int b) {
    for (int e = a; e < b; e++) {
      const int kid = kad_packer::find(P->label_key_id, S[su->sel_key[e]]);
      int vid = -1;
      if (kid >= 0) vid = kad_packer::find(P->label_vals[kid], S[su->sel_value[e]]);
      sel_code[e] = (kid < 0 || vid < 0) ? -1 : (((int64_t)kid << 32) | (uint32_t)vid);
    }
  });
  lap("selcodes");
  // toleration lists (parallel): a 64-bit content hash per unit, confirmed against the set's first unit
  auto& tol_hash = X.tol_hash;
  tol_hash.resize(W);
  parallel_for(W, threads, [&](int a, int b) {
    for (int w = a; w < b; w++) {
      uint64_t h = 1469598103934665603ull;
      for (int t = su->tol_off[w]; t < su->tol_off[w + 1]; t++)
        for (const int32_t s : {su->tol_key[t], su->tol_op[t], su->tol_value[t], su->tol_effect[t]}) {
          for (char ch : S[s]) h = (h ^ (uint8_t)ch) * 1099511628211ull;
          h = (h ^ 0x1ff) * 1099511628211ull;  // separator (not a byte value)
        }
      tol_hash[w] = h ^ (uint64_t)(su->tol_off[w + 1] - su->tol_off[w]);
    }
  });
  auto same_tols = [&](int a, int b) {
    const int na = su->tol_off[a + 1] - su->tol_off[a];
    if (na != su->tol_off[b + 1] - su->tol_off[b]) return false;
    for (int i = 0; i < na; i++) {
      const int ta = su->tol_off[a] + i, tb = su->tol_off[b] + i;
      if (S[su->tol_key[ta]] != S[su->tol_key[tb]] || S[su->tol_op[ta]] != S[su->tol_op[tb]] ||
          S[su->tol_value[ta]] != S[su->tol_value[tb]] || S[su->tol_effect[ta]] != S[su->tol_effect[tb]])
        return false;
    }
    return true;
  };

  lap("reqs");
  // ---- 2. interning in unit order (pack.py _Compiler.intern / tol_key), keys are views of stable words.
  // Batch-wide ids are the order of first occurrence over the units. In parallel: every chunk of units
  // interns into its own table (local ids in first-occurrence order within the chunk); the chunks' tables
  // are then merged in chunk order (only their distinct keys, serially), which assigns exactly the ids one
  // serial pass would; a last parallel pass rewrites the entries' local ids to batch-wide ones.
  static const int32_t kFalse[2] = {OP_FALSE, -1};
  auto words_sv = [](const int32_t* p, size_t n) { return sv(reinterpret_cast<const char*>(p), 4 * n); };
  auto& egid = X.egid;
  auto& fgid = X.fgid;
  auto& sgid = X.sgid;
  auto& tolset = X.tolset;
  egid.resize(R);
  fgid.resize(R);
  pfill(egid, (int32_t)-1);
  pfill(fgid, (int32_t)-1);
  sgid.resize((size_t)n_sel_total);
  tolset.resize(W);
  // chunks write the entries' local ids in place: an entry two units share (the column format allows it)
  // forces one chunk
  // (parallel: a compare-and-swap claims each entry for its unit; a second, different unit marks it shared)
  std::atomic<bool> shared{false};
  auto& owner = X.owner;  // the unit whose terms reference each requirement entry
  owner.resize(R);
  pfill(owner, (int32_t)-1);
  parallel_for(W, threads, [&](int a, int b) {
    auto own = [&](int e0, int e1, int w) {
      for (int e = e0; e < e1; e++) {
        int32_t prev = -1;
        if (!__atomic_compare_exchange_n(&owner[e], &prev, w, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED) && prev != w)
          shared.store(true, std::memory_order_relaxed);
      }
    };
    for (int w = a; w < b && !shared.load(std::memory_order_relaxed); w++) {
      for (int t = su->rterm_off[w]; t < su->rterm_off[w + 1]; t++)
        own(su->rt_req[t], su->rt_req[t] + su->rt_n_expr[t] + su->rt_n_field[t], w);
      for (int t = su->pterm_off[w]; t < su->pterm_off[w + 1]; t++) own(su->pt_req[t], su->pt_req[t] + su->pt_n_expr[t], w);
    }
  });
  const int NCH = shared ? 1 : std::max(1, std::min(threads, W));
  lap("owners");
  auto& chunks = X.chunks;
  if ((int)chunks.size() < NCH) chunks.resize(NCH);
  auto chunk_lo = [&](int c) { return (int)((int64_t)W * c / NCH); };
  parallel_for(NCH, NCH, [&](int ca, int cb) {
    for (int c = ca; c < cb; c++) {
      InternChunk& K = chunks[c];
      K.reset();
      auto intern = [&](sv w) -> int32_t {
        return K.req_ix.find_or_add(
            std::hash<sv>()(w), [&](int32_t x) { return K.reqs[x] == w; },
            [&] {
              K.reqs.push_back(w);
              return (int32_t)K.reqs.size() - 1;
            });
      };
      for (int w = chunk_lo(c); w < chunk_lo(c + 1); w++) {
        // toleration list → local set id (content identity: hash, confirmed against the set's first unit)
        tolset[w] = K.tol_ix.find_or_add(
            tol_hash[w], [&](int32_t x) { return same_tols(K.tol_rows[x], w); },
            [&] {
              K.tol_rows.push_back(w);
              return (int32_t)K.tol_rows.size() - 1;
            });
        // filter program: ClusterSelector entries, then required terms
        for (int64_t e = su->sel_off[w]; e < su->sel_off[w + 1]; e++) {
          const int64_t code = sel_code[e];
          if (code < 0) {
            sgid[e] = intern(words_sv(kFalse, 2));
            continue;
          }
          const int32_t x = K.eq_ix.find_or_add(
              (uint64_t)code, [&](int32_t y) { return K.eq_code[y] == code; },
              [&] {
                K.extra_words.push_back({OP_EQ | (1 << 8), (int32_t)(code >> 32), (int32_t)(uint32_t)code});
                K.eq_code.push_back(code);
                K.eq_req.push_back(intern(words_sv(K.extra_words.back().data(), 3)));
                return (int32_t)K.eq_code.size() - 1;
              });
          sgid[e] = K.eq_req[x];
        }
        const uint32_t f = su->flags[w];
        if ((f & KAD_SU_HAS_CLUSTER_AFFINITY) && (f & KAD_SU_HAS_REQUIRED)) {
          for (int t = su->rterm_off[w]; t < su->rterm_off[w + 1]; t++) {
            const int e0 = su->rt_req[t], e1 = e0 + su->rt_n_expr[t];
            bool ok = true;
            for (int e = e0; e < e1; e++) ok = ok && valid[e];
            if (e1 > e0 && ok)
              for (int e = e0; e < e1; e++)
                if (egid[e] < 0) egid[e] = intern(words_sv(wbuf.data() + eoff[e], elen[e]));
            const int g0 = e1, g1 = e1 + su->rt_n_field[t];
            bool fok = true;
            for (int e = g0; e < g1; e++) fok = fok && fvalid[e];
            if (g1 > g0 && fok)
              for (int e = g0; e < g1; e++)
                if (fgid[e] < 0) fgid[e] = intern(words_sv(fw.data() + 2 * (size_t)e, 2));
          }
        }
        // score program: preferred terms
        if (f & KAD_SU_HAS_CLUSTER_AFFINITY) {
          for (int t = su->pterm_off[w]; t < su->pterm_off[w + 1]; t++) {
            if (su->pt_weight[t] == 0) continue;
            const int e0 = su->pt_req[t], e1 = e0 + su->pt_n_expr[t];
            if (e1 == e0) continue;
            bool ok = true;
            for (int e = e0; e < e1; e++) ok = ok && valid[e];
            if (!ok) continue;
            for (int e = e0; e < e1; e++)
              if (egid[e] < 0) egid[e] = intern(words_sv(wbuf.data() + eoff[e], elen[e]));
          }
        }
      }
    }
  }, 1);
  lap("intern-A");
  // merge: batch-wide ids by first occurrence. The chunks' distinct keys, flattened in (chunk, local)
  // order, are split by hash over T threads; each thread (one flat index) finds the first occurrence of
  // every key of its share among equal keys, scanning in flat order; numbering the first occurrences
  // 0, 1, ... (a parallel prefix count) and giving every later occurrence its first's number yields the
  // ids of one serial pass over the units.
  auto first_occurrence = [&](int n_items, auto hash_of, auto same, std::vector<int32_t>& gid) -> int {
    auto& hs = X.fo_hash;
    auto& canon = X.fo_canon;
    hs.resize((size_t)n_items);
    canon.resize((size_t)n_items);
    gid.resize((size_t)n_items);
    parallel_for(n_items, threads, [&](int a, int b) {
      for (int g = a; g < b; g++) hs[g] = hash_of(g);
    });
    const int T = std::max(1, std::min(threads, 64));
    parallel_for(T, T, [&](int ta, int tb) {
      for (int t = ta; t < tb; t++) {
        FlatIndex ix;
        ix.reset((size_t)n_items / T + 16);
        for (int g = 0; g < n_items; g++) {
          if ((int)((FlatIndex::mix(hs[g]) >> 40) % (uint64_t)T) != t) continue;
          canon[g] = ix.find_or_add(hs[g], [&](int32_t x) { return same(x, g); }, [&] { return (int32_t)g; });
        }
      }
    }, 1);
    const int NB = std::max(1, std::min(threads * 4, (n_items + 4095) / 4096));
    std::vector<int32_t> cnt((size_t)NB + 1, 0);
    auto blo = [&](int k) { return (int)((int64_t)n_items * k / NB); };
    parallel_for(NB, threads, [&](int ka, int kb) {
      for (int k = ka; k < kb; k++) {
        int m = 0;
        for (int g = blo(k); g < blo(k + 1); g++) m += canon[g] == g;
        cnt[k + 1] = m;
      }
    }, 1);
    for (int k = 0; k < NB; k++) cnt[k + 1] += cnt[k];
    parallel_for(NB, threads, [&](int ka, int kb) {
      for (int k = ka; k < kb; k++) {
        int32_t next = cnt[k];
        for (int g = blo(k); g < blo(k + 1); g++)
          if (canon[g] == g) gid[g] = next++;
      }
    }, 1);
    parallel_for(n_items, threads, [&](int a, int b) {  // a later occurrence: its first's number
      for (int g = a; g < b; g++)
        if (canon[g] != g) gid[g] = gid[canon[g]];
    });
    return cnt[NB];
  };
  std::vector<int32_t> req_base((size_t)NCH + 1, 0), tol_base((size_t)NCH + 1, 0);
  for (int c = 0; c < NCH; c++) {
    req_base[c + 1] = req_base[c] + (int32_t)chunks[c].reqs.size();
    tol_base[c + 1] = tol_base[c] + (int32_t)chunks[c].tol_rows.size();
  }
  auto& flat_chunk = X.flat_chunk;
  flat_chunk.resize((size_t)std::max(req_base[NCH], tol_base[NCH]));
  auto fill_chunks = [&](const std::vector<int32_t>& base) {
    parallel_for(NCH, threads, [&](int ca, int cb) {
      for (int c = ca; c < cb; c++) std::fill(flat_chunk.begin() + base[c], flat_chunk.begin() + base[c + 1], c);
    }, 1);
  };
  fill_chunks(req_base);
  auto req_at = [&](int g) -> sv { const int c = flat_chunk[g]; return chunks[c].reqs[g - req_base[c]]; };
  auto& req_gid = X.req_gid;
  auto& tol_gid = X.tol_gid;
  const int NR0 = first_occurrence(
      req_base[NCH], [&](int g) { return (uint64_t)std::hash<sv>()(req_at(g)); },
      [&](int x, int y) { return req_at(x) == req_at(y); }, req_gid);
  std::vector<sv> reqs((size_t)NR0);  // by batch-wide id: the words as bytes (views into wbuf / fw / chunk words)
  parallel_for(req_base[NCH], threads, [&](int a, int b) {
    for (int g = a; g < b; g++)
      if (X.fo_canon[g] == g) reqs[req_gid[g]] = req_at(g);
  });
  fill_chunks(tol_base);
  auto tol_unit = [&](int g) { const int c = flat_chunk[g]; return chunks[c].tol_rows[g - tol_base[c]]; };
  const int NT0 = first_occurrence(
      tol_base[NCH], [&](int g) { return tol_hash[tol_unit(g)]; },
      [&](int x, int y) { return same_tols(tol_unit(x), tol_unit(y)); }, tol_gid);
  std::vector<int> tol_rows((size_t)NT0);  // first unit of each toleration set
  parallel_for(tol_base[NCH], threads, [&](int a, int b) {
    for (int g = a; g < b; g++)
      if (X.fo_canon[g] == g) tol_rows[tol_gid[g]] = tol_unit(g);
  });
  lap("merge");
  // local → batch-wide ids: units (toleration sets, selector entries) per chunk, requirement entries by
  // their owning unit's chunk
  auto& unit_chunk = X.unit_chunk;
  unit_chunk.resize(W);
  parallel_for(NCH, NCH, [&](int ca, int cb) {
    for (int c = ca; c < cb; c++) {
      const int32_t* rmap = req_gid.data() + req_base[c];
      const int32_t* tmap = tol_gid.data() + tol_base[c];
      for (int w = chunk_lo(c); w < chunk_lo(c + 1); w++) {
        unit_chunk[w] = c;
        tolset[w] = tmap[tolset[w]];
        for (int64_t e = su->sel_off[w]; e < su->sel_off[w + 1]; e++) sgid[e] = rmap[sgid[e]];
      }
    }
  }, 1);
  parallel_for(R, threads, [&](int a, int b) {
    for (int e = a; e < b; e++) {
      if (owner[e] < 0) continue;
      const int32_t* rmap = req_gid.data() + req_base[unit_chunk[owner[e]]];
      if (egid[e] >= 0) egid[e] = rmap[egid[e]];
      if (fgid[e] >= 0) fgid[e] = rmap[fgid[e]];
    }
  });
  const int NR = (int)reqs.size();
  const int NT = std::max(1, (int)tol_rows.size());
  lap("intern");

  // ---- 3. per-unit columns and CSR row lengths
  auto& flags = X.flags;
  auto& gvk = X.gvk;
  auto& n_sreq = X.n_sreq;
  auto& n_fp = X.n_fp;
  auto& n_sp = X.n_sp;
  auto& n_place = X.n_place;
  auto& n_cur = X.n_cur;
  auto& n_pref = X.n_pref;
  auto& n_key = X.n_key;
  auto& nr = X.nr;
  auto& maxc = X.maxc;
  auto& desired = X.desired;
  auto& out_len = X.out_len;
  for (auto* v : {&gvk, &n_sreq, &n_fp, &n_sp, &n_place, &n_cur, &n_pref, &n_key, &nr}) v->resize(W);
  flags.resize(W);
  maxc.resize(W);
  desired.resize(W);
  out_len.resize(W);
  // cluster names → snapshot ids, once per map / set entry; the name lookup itself once per string id of
  // the batch's table (a Go shim interns: the ~90 map entries per C4 unit name a few hundred clusters)
  auto cid_of = [&](int32_t id) {
    int32_t k = __atomic_load_n(&X.m_cid[id], __ATOMIC_RELAXED);
    if (!k) {
      k = kad_packer::find(P->name_id, S[id]) + 2;
      __atomic_store_n(&X.m_cid[id], k, __ATOMIC_RELAXED);
    }
    return k - 2;
  };
  auto resolve = [&](const int32_t* off, const int32_t* names, std::vector<int32_t>& ids) {
    const int n = W ? off[W] : 0;
    if (ids.size() < (size_t)n) ids.resize(n);  // every entry < n is written below
    parallel_for(n, threads, [&](int a, int b) {
      for (int i = a; i < b; i++) ids[i] = cid_of(names[i]);
    });
  };
  auto& place_c = X.place_c;
  auto& cur_c = X.cur_c;
  auto& wt_c = X.wt_c;
  auto& min_c = X.min_c;
  auto& max_c = X.max_c;
  auto& cap_c = X.cap_c;
  resolve(su->place_off, su->place_name, place_c);
  resolve(su->cur_off, su->cur_name, cur_c);
  resolve(su->wt_off, su->wt_name, wt_c);
  resolve(su->min_off, su->min_name, min_c);
  resolve(su->max_off, su->max_name, max_c);
  resolve(su->cap_off, su->cap_name, cap_c);
  lap("resolve");
  parallel_for(W, threads, [&](int a, int b) {
    std::vector<int32_t> ids;
    std::string gkey;
    IdSet set(C);
    int32_t lg = -1, lv = -1, lk = -1, lgvk = -1;  // the last (group, version, kind) string ids and their GVK id
    for (int w = a; w < b; w++) {
      const uint32_t sf = su->flags[w];
      uint32_t f = 0;
      if (sf & KAD_SU_DUPLICATE) f |= KAD_W_DUPLICATE;
      const int ncur_all = su->cur_off[w + 1] - su->cur_off[w];
      if ((sf & KAD_SU_STICKY) && ncur_all > 0) f |= KAD_W_STICKY;
      if (ncur_all > 0) f |= KAD_W_HAS_CURRENT;
      if (sf & KAD_SU_AVOID_DISRUPTION) f |= KAD_W_AVOID_DISRUPTION;
      const bool am = sf & KAD_SU_HAS_AUTO_MIGRATION;
      if (am && (sf & KAD_SU_KEEP_UNSCHED)) f |= KAD_W_KEEP_UNSCHED;
      desired[w] = 0;
      if (sf & KAD_SU_HAS_DESIRED) {
        f |= KAD_W_HAS_DESIRED;
        desired[w] = su->desired[w];
      }
      maxc[w] = 0;
      if (sf & KAD_SU_HAS_MAX_CLUSTERS) {
        f |= KAD_W_HAS_MAX_CLUSTERS;
        maxc[w] = su->max_clusters[w];
      }
      const int ns0 = su->scalar_off[w], ns1 = su->scalar_off[w + 1];
      if (!(su->req_cpu[w] == 0 && su->req_mem[w] == 0 && su->req_eph[w] == 0 && ns1 == ns0)) f |= KAD_W_FIT_NONZERO;
      int nsr = 0;
      for (int i = ns0; i < ns1; i++) nsr += su->scalar_val[i] > 0;
      n_sreq[w] = nsr;
      if (su->group[w] != lg || su->version[w] != lv || su->kind[w] != lk) {
        lg = su->group[w];
        lv = su->version[w];
        lk = su->kind[w];
        kad_packer::gvk_key(gkey, S[lg], S[lv], S[lk]);
        lgvk = kad_packer::find(P->gvk_id, gkey);
      }
      gvk[w] = lgvk;
      // filter program length and R_w
      int fl = 1 + (su->sel_off[w + 1] - su->sel_off[w]) + 1, rw = su->sel_off[w + 1] - su->sel_off[w];
      const bool ca = sf & KAD_SU_HAS_CLUSTER_AFFINITY;
      if (ca && (sf & KAD_SU_HAS_REQUIRED)) {
        fl += 1;
        for (int t = su->rterm_off[w]; t < su->rterm_off[w + 1]; t++) {
          const int e0 = su->rt_req[t], e1 = e0 + su->rt_n_expr[t];
          const int g0 = e1, g1 = e1 + su->rt_n_field[t];
          bool ok = true, fok = true;
          for (int e = e0; e < e1; e++) ok = ok && valid[e];
          for (int e = g0; e < g1; e++) fok = fok && fvalid[e];
          const int ne = (e1 > e0 && ok) ? e1 - e0 : 0, nf = (g1 > g0 && fok) ? g1 - g0 : 0;
          fl += 3 + ne + nf;
          rw += ne + nf;
        }
      }
      n_fp[w] = fl;
      // score program
      int sl = 1;
      bool serr = false;
      int64_t wsum = 0;
      if (ca) {
        for (int t = su->pterm_off[w]; t < su->pterm_off[w + 1]; t++) {
          if (su->pt_weight[t] == 0) continue;
          const int e0 = su->pt_req[t], e1 = e0 + su->pt_n_expr[t];
          if (e1 == e0) continue;
          bool ok = true;
          for (int e = e0; e < e1; e++) ok = ok && valid[e];
          if (!ok) {
            serr = true;
            continue;
          }
          sl += 2 + (e1 - e0);
          rw += e1 - e0;
          wsum += su->pt_weight[t] < 0 ? -(int64_t)su->pt_weight[t] : su->pt_weight[t];
        }
      }
      n_sp[w] = sl;
      nr[w] = rw;
      if (serr) f |= KAD_W_SCORE_ERROR;
      if (wsum > (1 << 20)) f |= KAD_W_WIDE_SCORES;
      // placement (a set: sorted unique snapshot ids)
      const int np_all = su->place_off[w + 1] - su->place_off[w];
      if (np_all > 0) f |= KAD_W_HAS_PLACEMENT;
      n_place[w] = (int)sorted_unique(place_c, su->place_off[w], su->place_off[w + 1], set, ids).size();
      int ncur = 0;
      for (int i = su->cur_off[w]; i < su->cur_off[w + 1]; i++) ncur += cur_c[i] >= 0;
      n_cur[w] = ncur;
      if (su->wt_off[w + 1] == su->wt_off[w]) f |= KAD_W_DYNAMIC_WEIGHTS;
      // preferences: union of the Weights / Min / Max / EstimatedCapacity (>= 0) names in the snapshot
      {
        int lo_id = INT32_MAX, hi_id = -1;
        size_t nn = 0;
        auto scan = [&](const std::vector<int32_t>& cs, const int32_t* off, const int64_t* val) {
          for (int i = off[w]; i < off[w + 1]; i++)
            if (cs[i] >= 0 && (!val || val[i] >= 0)) {
              lo_id = std::min(lo_id, cs[i]);
              hi_id = std::max(hi_id, cs[i]);
              nn++;
            }
        };
        scan(wt_c, su->wt_off, nullptr);
        scan(min_c, su->min_off, nullptr);
        scan(max_c, su->max_off, nullptr);
        if (am) scan(cap_c, su->cap_off, su->cap_val);
        auto each = [&](auto put) {
          auto one = [&](const std::vector<int32_t>& cs, const int32_t* off, const int64_t* val) {
            for (int i = off[w]; i < off[w + 1]; i++)
              if (cs[i] >= 0 && (!val || val[i] >= 0)) put(cs[i]);
          };
          one(wt_c, su->wt_off, nullptr);
          one(min_c, su->min_off, nullptr);
          one(max_c, su->max_off, nullptr);
          if (am) one(cap_c, su->cap_off, su->cap_val);
        };
        if (IdSet::worth(lo_id, hi_id, nn)) {
          each([&](int c) { set.add(c); });
          n_pref[w] = set.count_and_clear();
        } else {
          ids.clear();
          each([&](int c) { ids.push_back(c); });
          std::sort(ids.begin(), ids.end());
          n_pref[w] = (int)(std::unique(ids.begin(), ids.end()) - ids.begin());
        }
      }
      const size_t ln = S[su->name[w]].size(), lns = S[su->namespace_[w]].size();
      n_key[w] = (int)(lns ? lns + 1 + ln : ln);
      int64_t bound = C;
      if (select_max && (sf & KAD_SU_HAS_MAX_CLUSTERS) && maxc[w] >= 0 && maxc[w] < bound) bound = maxc[w];
      if (place_on && (f & KAD_W_HAS_PLACEMENT) && n_place[w] < bound) bound = n_place[w];
      if (f & KAD_W_STICKY) bound = 0;
      out_len[w] = bound;
      flags[w] = f;
    }
  });
  lap("units");

  // ---- layout (pack.py _assemble: header, then 256-B aligned arrays in enum order)
  auto csr_off = [&](const std::vector<int32_t>& len, std::vector<int32_t>& off) -> bool {
    off.resize((size_t)W + 1);
    off[0] = 0;
    int64_t acc = 0;
    for (int w = 0; w < W; w++) {
      acc += len[w];
      if (acc >= ((int64_t)1 << 31)) return false;
      off[w + 1] = (int32_t)acc;
    }
    return true;
  };
  auto& o_sreq = X.o_sreq;
  auto& o_fp = X.o_fp;
  auto& o_sp = X.o_sp;
  auto& o_place = X.o_place;
  auto& o_cur = X.o_cur;
  auto& o_pref = X.o_pref;
  auto& o_key = X.o_key;
  auto& o_out = X.o_out;
  o_out.resize((size_t)W + 1);
  int64_t max_row = 0;
  // the eight prefix sums are independent: one worker each
  bool csr_ok[7] = {true, true, true, true, true, true, true};
  {
    const std::vector<int32_t>* lens[7] = {&n_sreq, &n_fp, &n_sp, &n_place, &n_cur, &n_pref, &n_key};
    std::vector<int32_t>* offs[7] = {&o_sreq, &o_fp, &o_sp, &o_place, &o_cur, &o_pref, &o_key};
    parallel_for(8, threads, [&](int a, int b) {
      for (int q = a; q < b; q++) {
        if (q < 7) {
          csr_ok[q] = csr_off(*lens[q], *offs[q]);
          continue;
        }
        o_out[0] = 0;
        for (int w = 0; w < W; w++) {
          o_out[w + 1] = o_out[w] + out_len[w];
          max_row = std::max(max_row, out_len[w]);
        }
      }
    }, 1);
  }
  for (bool ok : csr_ok)
    if (!ok) return P->fail(KAD_EINVAL, "CSR array exceeds 2^31 entries; split the batch");
  lap("offsets");
  auto& req_off = X.req_off;
  req_off.resize((size_t)NR + 1);
  req_off[0] = 0;
  for (int r = 0; r < NR; r++) req_off[r + 1] = req_off[r] + (int32_t)(reqs[r].size() / 4);
  const size_t nS = (size_t)o_sreq[W], nF = (size_t)o_fp[W], nSP = (size_t)o_sp[W], nPL = (size_t)o_place[W],
               nC = (size_t)o_cur[W], nP = (size_t)o_pref[W], nK = (size_t)o_key[W], nRQ = (size_t)req_off[NR];
  // KAD_BATCH_NARROW_PREFS: every value of the input preference maps fits int32 (pack.py applies the same
  // rule to the same maps, so both packers choose the same layout)
  // The rule is checked where the values are read anyway: the rows pass below tests every input value (those
  // of entries it skips too) and, when one does not fit, the layout and rows are redone wide (a second pass
  // only for batches with out-of-range preference values).
  bool narrow = true;
  std::atomic<bool> wide_seen{false};
relayout:
  const size_t pv = narrow ? 4 : 8;  // bytes per preference value
  const size_t sizes[KAD_B_NARRAYS] = {
      4 * (size_t)W, 4 * (size_t)W, 8 * (size_t)W, 8 * (size_t)W, 8 * (size_t)W, 8 * (size_t)W, 4 * (size_t)W,
      8 * (size_t)NT * TW, 8 * (size_t)NT * TW,
      4 * ((size_t)W + 1), 4 * nS, 8 * nS,
      4 * ((size_t)W + 1), 4 * nF, 4 * ((size_t)W + 1), 4 * nSP,
      4 * ((size_t)W + 1), 4 * nPL, 4 * ((size_t)W + 1), 4 * nC, 8 * nC,
      4 * ((size_t)W + 1), 4 * nP, pv * nP, pv * nP, pv * nP, pv * nP, 4 * nP,
      4 * ((size_t)W + 1), nK, 8 * ((size_t)W + 1), 4 * ((size_t)NR + 1), 4 * nRQ};
  kad_batch_header h;
  std::memset(&h, 0, sizeof(h));
  size_t pos = align_up(sizeof(h));
  for (int i = 0; i < KAD_B_NARRAYS; i++) {
    h.off[i] = pos;
    pos += align_up(sizes[i]);
  }
  const size_t total = std::max(pos, (size_t)ALIGN);
  h.magic = KAD_BATCH_MAGIC;
  h.abi_version = KAD_ABI_VERSION;
  h.n_units = W;
  h.n_clusters = C;
  h.n_taint_words = TW;
  h.n_tolsets = NT;
  h.n_out_slots = o_out[W];
  h.max_row_slots = (int32_t)max_row;
  h.packed_filter_mask = prof->filter_mask;
  h.packed_select_plugin = prof->select_plugin;
  h.n_reqs = NR;
  h.flags = narrow ? KAD_BATCH_NARROW_PREFS : 0u;
  h.total_bytes = total;
  h.snapshot_fingerprint = P->fingerprint;
  uint8_t* base = P->reserve(total);
  if (!base) return P->fail(KAD_ENOMEM, "cannot allocate the batch blob");
  P->out_n = total;
  // every array is written in full below except the OR-filled toleration masks; zero those, the header
  // region and the alignment padding after each array (the blob must equal pack.py's byte for byte)
  std::memset(base, 0, h.off[0]);
  std::memcpy(base, &h, sizeof(h));
  for (int i = 0; i < KAD_B_NARRAYS; i++) {
    const size_t end = i + 1 < KAD_B_NARRAYS ? h.off[i + 1] : total;
    const size_t used = (i == KAD_B_TOL_ALL || i == KAD_B_TOL_PNS) ? 0 : sizes[i];
    std::memset(base + h.off[i] + used, 0, end - h.off[i] - used);
  }
  auto A = [&](int i) { return base + h.off[i]; };
  {
    // the per-unit arrays, copied in parallel pieces of <= 4 MiB
    struct Put {
      int i;
      const void* src;
      size_t n;
    };
    const Put puts[] = {{KAD_B_FLAGS, flags.data(), 4 * (size_t)W}, {KAD_B_GVK, gvk.data(), 4 * (size_t)W},
                        {KAD_B_REQ_CPU, su->req_cpu, 8 * (size_t)W}, {KAD_B_REQ_MEM, su->req_mem, 8 * (size_t)W},
                        {KAD_B_DESIRED, desired.data(), 8 * (size_t)W}, {KAD_B_MAX_CLUSTERS, maxc.data(), 8 * (size_t)W},
                        {KAD_B_TOLSET, tolset.data(), 4 * (size_t)W},
                        {KAD_B_SREQ_OFF, o_sreq.data(), 4 * ((size_t)W + 1)}, {KAD_B_FPROG_OFF, o_fp.data(), 4 * ((size_t)W + 1)},
                        {KAD_B_SPROG_OFF, o_sp.data(), 4 * ((size_t)W + 1)}, {KAD_B_PLACE_OFF, o_place.data(), 4 * ((size_t)W + 1)},
                        {KAD_B_CUR_OFF, o_cur.data(), 4 * ((size_t)W + 1)}, {KAD_B_PREF_OFF, o_pref.data(), 4 * ((size_t)W + 1)},
                        {KAD_B_KEY_OFF, o_key.data(), 4 * ((size_t)W + 1)}, {KAD_B_OUT_OFF, o_out.data(), 8 * ((size_t)W + 1)},
                        {KAD_B_REQ_OFF, req_off.data(), 4 * ((size_t)NR + 1)}};
    constexpr size_t PIECE = 4u << 20;
    std::vector<std::array<size_t, 3>> pieces;  // put, offset, length
    for (size_t q = 0; q < sizeof(puts) / sizeof(puts[0]); q++)
      for (size_t o = 0; o < puts[q].n; o += PIECE) pieces.push_back({q, o, std::min(PIECE, puts[q].n - o)});
    parallel_for((int)pieces.size(), threads, [&](int a, int b) {
      for (int x = a; x < b; x++) {
        const Put& pu = puts[pieces[x][0]];
        std::memcpy(A(pu.i) + pieces[x][1], static_cast<const uint8_t*>(pu.src) + pieces[x][1], pieces[x][2]);
      }
    }, 1);
  }
  {
    int32_t* rq = reinterpret_cast<int32_t*>(A(KAD_B_REQ));
    parallel_for(NR, threads, [&](int a, int b) {
      for (int r = a; r < b; r++) std::memcpy(rq + req_off[r], reqs[r].data(), reqs[r].size());
    });
  }

  lap("layout");
  // ---- 4. CSR rows in place
  int32_t* sreq_id = reinterpret_cast<int32_t*>(A(KAD_B_SREQ_ID));
  int64_t* sreq_val = reinterpret_cast<int64_t*>(A(KAD_B_SREQ_VAL));
  int32_t* fprog = reinterpret_cast<int32_t*>(A(KAD_B_FPROG));
  int32_t* sprog = reinterpret_cast<int32_t*>(A(KAD_B_SPROG));
  int32_t* place = reinterpret_cast<int32_t*>(A(KAD_B_PLACE));
  int32_t* cur_id = reinterpret_cast<int32_t*>(A(KAD_B_CUR_ID));
  int64_t* cur_rep = reinterpret_cast<int64_t*>(A(KAD_B_CUR_REP));
  int32_t* pref_id = reinterpret_cast<int32_t*>(A(KAD_B_PREF_ID));
  uint8_t* const pref_col[4] = {A(KAD_B_PREF_W), A(KAD_B_PREF_MIN), A(KAD_B_PREF_MAX), A(KAD_B_PREF_CAP)};
  // entry j's weight, min, max, capacity, in the batch's width
  auto put_pref = [&](int64_t j, int64_t wv, int64_t mn, int64_t mx, int64_t cp) {
    const int64_t v[4] = {wv, mn, mx, cp};
    for (int q = 0; q < 4; q++) {
      if (narrow) reinterpret_cast<int32_t*>(pref_col[q])[j] = (int32_t)v[q];
      else reinterpret_cast<int64_t*>(pref_col[q])[j] = v[q];
    }
  };
  uint32_t* pref_fl = reinterpret_cast<uint32_t*>(A(KAD_B_PREF_FLAGS));
  uint8_t* keyb = A(KAD_B_KEY);
  struct PrefEntry {
    int32_t c, m, i;
  };
  auto fits32 = [](int64_t v) { return v >= INT32_MIN && v <= INT32_MAX; };
  parallel_for(W, threads, [&](int a, int b) {
    bool wide = false;  // an input value of this range outside int32 (the narrow rule)
    std::vector<int32_t> ids;
    std::vector<std::pair<int32_t, int64_t>> cl;
    std::vector<PrefEntry> pe;
    IdSet set(C);
    // dense per-cluster merge of the four preference maps (small snapshots): values and a map-present mask
    const bool dense = C <= (1 << 16);
    std::vector<int64_t> dv(dense ? 4 * (size_t)C : 0);
    std::vector<uint8_t> dm(dense ? (size_t)C : 0, 0);
    for (int w = a; w < b; w++) {
      const uint32_t sf = su->flags[w];
      // scalar requests with value > 0, in map order (snapshot id or -1)
      int k = o_sreq[w];
      for (int i = su->scalar_off[w]; i < su->scalar_off[w + 1]; i++)
        if (su->scalar_val[i] > 0) {
          sreq_id[k] = kad_packer::find(P->scalar_id, S[su->scalar_name[i]]);
          sreq_val[k++] = su->scalar_val[i];
        }
      // filter program (kad_sched.h predicate programs)
      int32_t* fp = fprog + o_fp[w];
      int pc = 0;
      fp[pc++] = su->sel_off[w + 1] - su->sel_off[w];
      for (int64_t e = su->sel_off[w]; e < su->sel_off[w + 1]; e++) fp[pc++] = sgid[e];
      const bool ca = sf & KAD_SU_HAS_CLUSTER_AFFINITY;
      if (!(ca && (sf & KAD_SU_HAS_REQUIRED))) {
        fp[pc++] = 0;
      } else {
        fp[pc++] = 1;
        fp[pc++] = su->rterm_off[w + 1] - su->rterm_off[w];
        for (int t = su->rterm_off[w]; t < su->rterm_off[w + 1]; t++) {
          const int e0 = su->rt_req[t], e1 = e0 + su->rt_n_expr[t];
          const int g0 = e1, g1 = e1 + su->rt_n_field[t];
          bool ok = true, fok = true;
          for (int e = e0; e < e1; e++) ok = ok && valid[e];
          for (int e = g0; e < g1; e++) fok = fok && fvalid[e];
          int tf = 0;
          if (e1 > e0) tf |= KAD_TERM_HAS_EXPR | (ok ? KAD_TERM_EXPR_VALID : 0);
          if (g1 > g0) tf |= KAD_TERM_HAS_FIELD | (fok ? KAD_TERM_FIELD_VALID : 0);
          const int ne = (e1 > e0 && ok) ? e1 - e0 : 0, nf = (g1 > g0 && fok) ? g1 - g0 : 0;
          fp[pc++] = tf;
          fp[pc++] = ne;
          fp[pc++] = nf;
          for (int e = 0; e < ne; e++) fp[pc++] = egid[e0 + e];
          for (int e = 0; e < nf; e++) fp[pc++] = fgid[g0 + e];
        }
      }
      // score program
      int32_t* sp = sprog + o_sp[w];
      int sc = 1, nt = 0;
      if (ca) {
        for (int t = su->pterm_off[w]; t < su->pterm_off[w + 1]; t++) {
          if (su->pt_weight[t] == 0) continue;
          const int e0 = su->pt_req[t], e1 = e0 + su->pt_n_expr[t];
          if (e1 == e0) continue;
          bool ok = true;
          for (int e = e0; e < e1; e++) ok = ok && valid[e];
          if (!ok) continue;
          sp[sc++] = su->pt_weight[t];
          sp[sc++] = e1 - e0;
          for (int e = e0; e < e1; e++) sp[sc++] = egid[e];
          nt++;
        }
      }
      sp[0] = nt;
      // placement
      sorted_unique(place_c, su->place_off[w], su->place_off[w + 1], set, ids);
      if (!ids.empty()) std::memcpy(place + o_place[w], ids.data(), 4 * ids.size());
      // current clusters (nil replicas → DesiredReplicas, rsp.go:119-126), by snapshot id
      cl.clear();
      const int64_t tot = (sf & KAD_SU_HAS_DESIRED) ? su->desired[w] : 0;
      for (int i = su->cur_off[w]; i < su->cur_off[w + 1]; i++)
        if (cur_c[i] >= 0) cl.emplace_back(cur_c[i], su->cur_has_rep[i] ? su->cur_rep[i] : tot);
      std::sort(cl.begin(), cl.end());
      for (size_t i = 0; i < cl.size(); i++) {
        cur_id[o_cur[w] + i] = cl[i].first;
        cur_rep[o_cur[w] + i] = cl[i].second;
      }
      // preferences sorted by snapshot id: (cluster, map, entry) triples, merged per cluster;
      // a repeated map key keeps its last entry, as a Go map holds one
      const bool am = sf & KAD_SU_HAS_AUTO_MIGRATION;
      if (dense) {  // maps in order, entries in order: a repeated key's last entry wins, as in the sort below
        auto put = [&](int c, int m, int64_t v) {
          dv[(size_t)m * C + c] = v;
          dm[c] |= (uint8_t)(1u << m);
          set.add(c);
        };
        for (int i = su->wt_off[w]; i < su->wt_off[w + 1]; i++) {
          wide |= !fits32(su->wt_val[i]);
          if (wt_c[i] >= 0) put(wt_c[i], 0, su->wt_val[i]);
        }
        for (int i = su->min_off[w]; i < su->min_off[w + 1]; i++) {
          wide |= !fits32(su->min_val[i]);
          if (min_c[i] >= 0) put(min_c[i], 1, su->min_val[i]);
        }
        for (int i = su->max_off[w]; i < su->max_off[w + 1]; i++) {
          wide |= !fits32(su->max_val[i]);
          if (max_c[i] >= 0) put(max_c[i], 2, su->max_val[i]);
        }
        if (am)
          for (int i = su->cap_off[w]; i < su->cap_off[w + 1]; i++) {
            wide |= !fits32(su->cap_val[i]);
            if (cap_c[i] >= 0 && su->cap_val[i] >= 0) put(cap_c[i], 3, su->cap_val[i]);
          }
        int j = o_pref[w];
        set.drain([&](int c) {
          const uint8_t m = dm[c];
          dm[c] = 0;
          pref_id[j] = c;
          put_pref(j, (m & 1) ? dv[c] : 0, (m & 2) ? dv[(size_t)C + c] : 0, (m & 4) ? dv[2 * (size_t)C + c] : 0,
                   (m & 8) ? dv[3 * (size_t)C + c] : 0);
          pref_fl[j] = ((m & 1) ? KAD_PREF_HAS_WEIGHT : 0u) | ((m & 4) ? KAD_PREF_HAS_MAX : 0u) |
                       ((m & 8) ? KAD_PREF_HAS_CAP : 0u);
          j++;
        });
      } else {
      pe.clear();
      for (int i = su->wt_off[w]; i < su->wt_off[w + 1]; i++) wide |= !fits32(su->wt_val[i]);
      for (int i = su->min_off[w]; i < su->min_off[w + 1]; i++) wide |= !fits32(su->min_val[i]);
      for (int i = su->max_off[w]; i < su->max_off[w + 1]; i++) wide |= !fits32(su->max_val[i]);
      if (am)
        for (int i = su->cap_off[w]; i < su->cap_off[w + 1]; i++) wide |= !fits32(su->cap_val[i]);
      for (int i = su->wt_off[w]; i < su->wt_off[w + 1]; i++)
        if (wt_c[i] >= 0) pe.push_back({wt_c[i], 0, i});
      for (int i = su->min_off[w]; i < su->min_off[w + 1]; i++)
        if (min_c[i] >= 0) pe.push_back({min_c[i], 1, i});
      for (int i = su->max_off[w]; i < su->max_off[w + 1]; i++)
        if (max_c[i] >= 0) pe.push_back({max_c[i], 2, i});
      if (am)
        for (int i = su->cap_off[w]; i < su->cap_off[w + 1]; i++)
          if (cap_c[i] >= 0 && su->cap_val[i] >= 0) pe.push_back({cap_c[i], 3, i});
      std::sort(pe.begin(), pe.end(), [](const PrefEntry& x, const PrefEntry& y) {
        return x.c != y.c ? x.c < y.c : (x.m != y.m ? x.m < y.m : x.i < y.i);
      });
      int j = o_pref[w];
      for (size_t q = 0; q < pe.size();) {
        const int c = pe[q].c;
        int64_t wv = 0, mn = 0, mx = 0, cp = 0;
        uint32_t fl = 0;
        for (; q < pe.size() && pe[q].c == c; q++) {
          const int i = pe[q].i;
          switch (pe[q].m) {
            case 0: wv = su->wt_val[i]; fl |= KAD_PREF_HAS_WEIGHT; break;
            case 1: mn = su->min_val[i]; break;
            case 2: mx = su->max_val[i]; fl |= KAD_PREF_HAS_MAX; break;
            default: cp = su->cap_val[i]; fl |= KAD_PREF_HAS_CAP; break;
          }
        }
        pref_id[j] = c;
        put_pref(j, wv, mn, mx, cp);
        pref_fl[j] = fl;
        j++;
      }
      }
      // su.Key()
      uint8_t* kb = keyb + o_key[w];
      const sv nsp = S[su->namespace_[w]], nm = S[su->name[w]];
      if (!nsp.empty()) {
        std::memcpy(kb, nsp.data(), nsp.size());
        kb[nsp.size()] = '/';
        kb += nsp.size() + 1;
      }
      if (!nm.empty()) std::memcpy(kb, nm.data(), nm.size());
    }
    if (wide) wide_seen.store(true, std::memory_order_relaxed);
  });

  lap("rows");
  if (narrow && wide_seen.load()) {
    narrow = false;
    goto relayout;
  }
  // tolerated-taint masks per toleration set (framework/util.go:406-450 via Toleration.ToleratesTaint)
  uint64_t* tol_all = reinterpret_cast<uint64_t*>(A(KAD_B_TOL_ALL));
  uint64_t* tol_pns = reinterpret_cast<uint64_t*>(A(KAD_B_TOL_PNS));
  const int ntaint = (int)P->taint_key.size();
  // taint ids by key (a toleration with a key only tolerates taints of that key; an empty key, every taint)
  std::unordered_map<sv, std::vector<int32_t>> taints_of_key;
  std::vector<int32_t> all_taints(ntaint);
  for (int tid = 0; tid < ntaint; tid++) {
    taints_of_key[sv(P->taint_key[tid])].push_back(tid);
    all_taints[tid] = tid;
  }
  parallel_for((int)tol_rows.size(), threads, [&](int a, int b) {
    for (int r = a; r < b; r++) {
      const int w = tol_rows[r];
      uint64_t* ta = tol_all + (size_t)r * TW;
      uint64_t* tp = tol_pns + (size_t)r * TW;
      for (int t = su->tol_off[w]; t < su->tol_off[w + 1]; t++) {
        const sv key = S[su->tol_key[t]], op = S[su->tol_op[t]], val = S[su->tol_value[t]], eff = S[su->tol_effect[t]];
        const bool equal = op.empty() || op == "Equal";
        if (!equal && op != "Exists") continue;  // tolerates nothing
        const std::vector<int32_t>* cand = &all_taints;
        if (!key.empty()) {
          auto it = taints_of_key.find(key);
          if (it == taints_of_key.end()) continue;
          cand = &it->second;
        }
        const bool pns = eff.empty() || eff == "PreferNoSchedule";
        for (const int32_t tid : *cand) {
          if (!eff.empty() && eff != P->taint_effect[tid]) continue;
          if (equal && val != P->taint_value[tid]) continue;
          const uint64_t bit = 1ull << (tid % 64);
          ta[tid / 64] |= bit;
          if (pns) tp[tid / 64] |= bit;
        }
      }
    }
  });

  lap("tolsets");
  if (stats) {
    if (stats->n_reqs) std::memcpy(stats->n_reqs, nr.data(), 4 * (size_t)W);
    if (stats->n_tols)
      for (int w = 0; w < W; w++) stats->n_tols[w] = su->tol_off[w + 1] - su->tol_off[w];
    stats->n_distinct_reqs = NR;
    stats->n_tolsets = NT;
  }
  *nbytes = total;
  return KAD_OK;
}

// The entry points: nothing may unwind through the C ABI. An exception out of the packer (std::bad_alloc
// from a task's vectors, rethrown by the worker pool after every worker has finished) becomes KAD_ENOMEM.
int kad_packer_create(const kad_pack_vocab* v, kad_packer** out) {
  try {
    return packer_create_impl(v, out);
  } catch (const std::exception& e) {
    g_create_err = std::string("packer creation failed: ") + e.what();
    return KAD_ENOMEM;
  }
}

int kad_packer_take(kad_packer* p, void* dst, size_t cap) {
  try {
    return packer_take_impl(p, dst, cap);
  } catch (const std::exception& e) {
    return p->fail(KAD_ENOMEM, std::string("copy-out failed: ") + e.what());
  }
}

int kad_pack_batch(kad_packer* P, const kad_profile* prof, const kad_su_columns* su, int threads, size_t* nbytes,
                   kad_pack_stats* stats) {
  try {
    return pack_batch_impl(P, prof, su, threads, nbytes, stats);
  } catch (const std::exception& e) {
    if (!P) return KAD_ENOMEM;
    return P->fail(KAD_ENOMEM, std::string("packing failed: ") + e.what());
  }
}

}  // extern "C"
