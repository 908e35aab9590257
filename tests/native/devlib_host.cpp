// TEST ONLY: compiles the kernels' per-thread routines (zeebe_amd/csrc/zb_devlib.hpp) for the host so
// that their byte-level logic can be fuzzed against the oracle on CPU (tests/test_devlib_host.py).
// Nothing here is part of the product; the product runs these routines only inside the HIP kernels.
#include <cstdint>
#include <cstdio>
#include <cstring>
#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __global__
static inline float __uint_as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static inline double __longlong_as_double(long long u) { double d; std::memcpy(&d, &u, 8); return d; }
#define HIP_INCLUDE_HIP_HIP_RUNTIME_H
#include "../../zeebe_amd/csrc/zb_devlib.hpp"
#include "../../zeebe_amd/csrc/zb_xmerge.hpp"
#include "../../zeebe_amd/csrc/zb_model.cpp"  // the product's deploy-time compilers (json-path, mapping targets)

#include <string>
#include <vector>

using namespace zbg;

// the exact tree's string chunks read up to 7 bytes past a document (the device arena keeps ARENA_SLACK readable bytes
// past its end): documents from Python are copied into padded buffers
static std::vector<uint8_t> padded(const uint8_t* p, uint32_t n) {
  std::vector<uint8_t> v(n + 64, 0);
  if (n) std::memcpy(v.data(), p, n);
  return v;
}

extern "C" {
// returns length, -1 malformed, -2 unsupported
long devlib_merge(const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt, uint8_t* out, uint32_t cap) {
  Out o{nullptr, 0};
  bool unsup = false;
  if (!merge_docs(src, ns, tgt, nt, o, unsup)) return -1;
  if (unsup) return -2;
  if (o.n > cap) return -3;
  Out w{out, 0};
  bool u2 = false;
  merge_docs(src, ns, tgt, nt, w, u2);
  if (w.n != o.n) return -4;
  return (long)w.n;
}
// flat fast path: returns length, -5 when the documents are not flat (caller would use merge_docs)
long devlib_merge_flat(const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt, uint8_t* out, uint32_t cap) {
  uint32_t n = 0;
  if (!merge_flat(src, ns, tgt, nt, out, cap, n)) return -5;
  return (long)n;
}
// explicit io-mappings: map_documents over caller-built tables (tgt == nullptr: extract). Returns the
// output length, or -(10 + status) for a MAP_* status other than MAP_OK (fail_query in *fq).
long devlib_map(const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt, const DevMapping* maps,
                uint32_t nmaps, const DevSeg* segs, const DevQuery* queries, const DevFilter* filters,
                const uint8_t* pool, uint8_t* out, uint32_t cap, uint32_t* fq) {
  static MNode ws[MAP_NODES];
  uint16_t q = 0xffff;
  Out o{nullptr, 0};
  int st = map_documents(src, ns, tgt, nt, maps, nmaps, segs, queries, filters, pool, ws, o, q);
  *fq = q;
  if (st != MAP_OK) return -(10 + st);
  if (o.n > cap) return -3;
  Out w{out, 0};
  st = map_documents(src, ns, tgt, nt, maps, nmaps, segs, queries, filters, pool, ws, w, q);
  if (st != MAP_OK || w.n != o.n) return -4;
  return (long)w.n;
}
// the same through the product's deploy-time compilers: spec = "source\ttarget\n"...; -20 = compile error (err)
long devlib_map_text(const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt, const char* spec, uint8_t* out,
                     uint32_t cap, uint32_t* fq, char* err, uint32_t errcap) {
  ModelTables t;
  std::string sp(spec), e;
  size_t p = 0;
  while (p < sp.size()) {
    size_t tab = sp.find('\t', p), nl = sp.find('\n', p);
    if (tab == std::string::npos || nl == std::string::npos || tab > nl) return -21;
    if (compile_mapping(t, sp.substr(p, tab - p), sp.substr(tab + 1, nl - tab - 1), e) < 0) {
      snprintf(err, errcap, "%s", e.c_str());
      return -20;
    }
    p = nl + 1;
  }
  if (t.pool.empty()) t.pool.push_back(0);
  return devlib_map(src, ns, tgt, nt, t.maps.data(), (uint32_t)t.maps.size(), t.segs.data(), t.queries.data(),
                    t.filters.data(), t.pool.data(), out, cap, fq);
}
// returns count of results; first result pos/len in out[0..1]; -1 unsupported
long devlib_query(const uint8_t* doc, uint32_t n, const uint8_t* f_ids, const int32_t* f_idx,
                  const uint8_t* keys, const uint32_t* key_off, const uint32_t* key_len, uint32_t nf, int fast,
                  uint32_t* out) {
  DevFilter fs[32];
  for (uint32_t i = 0; i < nf; i++) {
    fs[i] = DevFilter{};
    fs[i].id = f_ids[i];
    fs[i].index = f_idx[i];
    fs[i].key_off = key_off[i];
    fs[i].key_len = (uint16_t)key_len[i];
  }
  QueryResult r;
  bool ok = fast ? query_fast(doc, n, keys + fs[1].key_off, fs[1].key_len, r)
                 : query_general(doc, n, fs, nf, keys, r);
  if (!ok) return -1;
  out[0] = r.pos;
  out[1] = r.len;
  return r.count;
}
// the product's json-path compiler (zb_model.cpp compile_filters, JsonPathQueryCompiler): the filter instances
// (filter id, index) -- #instances, or -1 with the error reason
long devlib_compile_path(const char* expr, int32_t* ids, int32_t* idx, uint32_t cap, char* err, uint32_t errcap) {
  ModelTables t;
  std::vector<DevFilter> fs;
  std::string e;
  if (!compile_filters(expr, fs, t, e)) {
    snprintf(err, errcap, "%s", e.c_str());
    return -1;
  }
  for (uint32_t i = 0; i < fs.size() && i < cap; i++) { ids[i] = fs[i].id; idx[i] = fs[i].index; }
  return (long)fs.size();
}
// a json-path compiled by the product's compiler (compile_query) and run by the kernels' query entry (run_query, the
// one k_subscribe and the condition VM use): #results, first result in out[0..1]; -1 unsupported, -20 invalid path
long devlib_query_text(const char* expr, const uint8_t* doc, uint32_t n, uint32_t* out) {
  ModelTables t;
  std::string e;
  const int q = compile_query(t, expr, e);
  if (q < 0) return -20;
  if (t.pool.empty()) t.pool.push_back(0);
  QueryResult r;
  if (!run_query(doc, n, t.queries[q], t.filters.data(), t.pool.data(), r)) return -1;
  out[0] = r.pos;
  out[1] = r.len;
  return r.count;
}
// read_tok (the kernels' MsgPackReader.readToken): out = type (TokType), boolean, size / length, header length,
// bytes consumed; 0, or -1 when the token does not read
long devlib_read_token(const uint8_t* p, uint32_t n, int64_t* ival, double* fval, int32_t* out) {
  Tok t;
  if (!read_tok(p, n, t)) return -1;
  *ival = t.ival;
  *fval = t.fval;
  out[0] = t.type; out[1] = t.bval ? 1 : 0; out[2] = (int32_t)t.len; out[3] = t.hdr; out[4] = (int32_t)t.total;
  return 0;
}
// The exact tree (zb_xmerge.hpp) as built for a document -- indexed (mode 0: MsgPackDocumentIndexer.index) or
// extracted by mappings (mode 1: MsgPackDocumentExtractor.extract, spec as devlib_map_text) -- dumped as one line per
// typed node: type (M map, A array, L existing leaf, X extracted leaf), NUL, id, NUL, children joined by 0x1e in
// insertion order, NUL, leaf bytes (hex; empty: no leaf), '\n'. Returns the dump length, or -(100 + X_* status).
long devlib_xtree_dump(const uint8_t* doc0, uint32_t n, const char* spec, int mode, char* out, uint32_t cap) {
  static uint8_t slab[XSLAB_BYTES];
  const std::vector<uint8_t> dv = padded(doc0, n);
  const uint8_t* doc = dv.data();
  XTree T;
  int st;
  if (mode == 0) {
    if (!T.init(XWs{slab, XSLAB_BYTES, 0, 1}, x_tokens(doc, n))) return -(100 + T.status);
    T.index(0, doc, n, false);
    st = T.status;
  } else {
    ModelTables t;
    std::string sp(spec), e;
    size_t p = 0;
    while (p < sp.size()) {
      size_t tab = sp.find('\t', p), nl = sp.find('\n', p);
      if (tab == std::string::npos || nl == std::string::npos || tab > nl) return -21;
      if (compile_mapping(t, sp.substr(p, tab - p), sp.substr(tab + 1, nl - tab - 1), e) < 0) return -20;
      p = nl + 1;
    }
    if (t.pool.empty()) t.pool.push_back(0);
    uint16_t q = 0xffff;
    st = x_map_tree(T, XWs{slab, XSLAB_BYTES, 0, 1}, doc, n, nullptr, 0, t.maps.data(), (uint32_t)t.maps.size(), t.segs.data(),
                    t.queries.data(), t.filters.data(), t.pool.data(), q);
  }
  if (st != X_OK) return -(100 + st);
  std::string d;
  static const char HEX[] = "0123456789abcdef";
  for (uint32_t i = 0; i < T.nn; i++) {
    const XNode& x = T.nodes[i];
    if (x.tree != 0 || x.type == XT_NONE) continue;
    d += x.type == XT_MAP ? 'M' : x.type == XT_ARRAY ? 'A' : x.type == XT_EXTRACTED_LEAF ? 'X' : 'L';
    d += '\0';
    d.append((const char*)T.s(x.id), x.id.len);
    d += '\0';
    if (x.has_childs)
      for (uint32_t c = x.cfirst; c != XNONE; c = T.ch[c].next) {
        if (c != x.cfirst) d += '\x1e';
        d.append((const char*)T.s(T.ch[c].name), T.ch[c].name.len);
      }
    d += '\0';
    if (x.has_leaf)  // (extracted and indexed leaves both come from the one document here)
      for (uint32_t k = 0; k < x.llen; k++) { d += HEX[doc[x.lpos + k] >> 4]; d += HEX[doc[x.lpos + k] & 15]; }
    d += '\n';
  }
  if (d.size() <= cap) memcpy(out, d.data(), d.size());
  return (long)d.size();
}
// the exact tree (zb_xmerge.hpp): x_merge, or x_map over the product's compiled mappings (spec as devlib_map_text,
// empty spec = merge). Returns the output length, or -(100 + X_* status) (fail_query in *fq), -20 compile error.
// lane < 0: one slab of its own (the kernels' big slabs); lane 0..63: lane `lane` of an interleaved group of 64
// XLANE_BYTES workspaces (the kernels' lane workspaces, zb_xlock.hpp x_run) -- X_UNSUP when the pair does not fit it
long devlib_xmerge(const uint8_t* src0, uint32_t ns, const uint8_t* tgt0, uint32_t nt, const char* spec, int extract,
                   uint8_t* out, uint32_t cap, uint32_t* fq, char* err, uint32_t errcap, int lane) {
  static uint8_t slab[XSLAB_BYTES];
  static std::vector<uint8_t> group;
  if (lane >= 0 && group.empty()) group.assign((size_t)64 * XLANE_BYTES, 0xA5);
  const XWs ws = lane < 0 ? XWs{slab, XSLAB_BYTES, 0, 1} : XWs{group.data(), XLANE_BYTES, (uint32_t)lane, 64};
  const std::vector<uint8_t> sv = padded(src0, ns), tv = padded(tgt0, nt);
  const uint8_t* src = sv.data();
  const uint8_t* tgt = tv.data();
  ModelTables t;
  std::string sp(spec), e;
  size_t p = 0;
  while (p < sp.size()) {
    size_t tab = sp.find('\t', p), nl = sp.find('\n', p);
    if (tab == std::string::npos || nl == std::string::npos || tab > nl) return -21;
    if (compile_mapping(t, sp.substr(p, tab - p), sp.substr(tab + 1, nl - tab - 1), e) < 0) {
      snprintf(err, errcap, "%s", e.c_str());
      return -20;
    }
    p = nl + 1;
  }
  if (t.pool.empty()) t.pool.push_back(0);
  Out o{out, 0};
  uint16_t q = 0xffff;
  int st;
  if (t.maps.empty())
    st = x_merge(ws, src, ns, tgt, nt, o, cap);
  else
    st = x_map(ws, src, ns, extract ? nullptr : tgt, nt, t.maps.data(), (uint32_t)t.maps.size(),
               t.segs.data(), t.queries.data(), t.filters.data(), t.pool.data(), o, cap, q);
  *fq = q;
  if (st != X_OK) return -(100 + st);
  return (long)o.n;
}
}
