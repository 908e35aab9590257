// zb_devlib.hpp — per-thread msgpack, json-path, json-el and merge routines for the gfx950 kernels.
//
// Semantics follow the reference exactly where the hot path observes them:
//   token reading:     msgpack-core/.../spec/MsgPackReader.java:302-345 (readToken)
//   query executor:    json-path/.../query/MsgPackQueryExecutor.java:60-144 (full traversal, no early exit)
//   condition types:   json-el/.../JsonConditionInterpreter.java:138-240
//   default merge:     json-path/.../mapping/{MsgPackDocumentIndexer,MsgPackTree,MsgPackDocumentTreeWriter}.java
// Shapes the kernels do not implement set DE_UNSUPPORTED instead of guessing.
#pragma once
#include <hip/hip_runtime.h>

#include "zb_device.hpp"

namespace zbg {

// the msgpack / json-path readers also build for the host (tests/xmerge_host.cpp runs the exact merge there)
#define ZB_HD __host__ __device__

// ------------------------------------------------------------------------------ msgpack reading
struct Tok {
  uint8_t type;      // TokType
  uint8_t hdr;       // header length
  uint32_t len;      // str/bin payload length, map entries / array elements
  uint32_t total;    // header + payload (containers: header only)
  int64_t ival;
  double fval;
  bool bval;
};

ZB_HD __forceinline__ uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
ZB_HD __forceinline__ uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
ZB_HD __forceinline__ uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }

// Reads the token at p (n bytes available). Returns false on malformed / unsupported input.
ZB_HD inline bool read_tok(const uint8_t* p, uint32_t n, Tok& t) {
  if (n == 0) return false;
  uint8_t b = p[0];
  t.hdr = 1; t.len = 0; t.ival = 0; t.fval = 0; t.bval = false;
  if (b <= 0x7f || b >= 0xe0) { t.type = TT_INTEGER; t.ival = (int8_t)b; t.total = 1; return true; }
  if ((b & 0xf0) == 0x80) { t.type = TT_MAP; t.len = b & 0x0f; t.total = 1; return true; }
  if ((b & 0xf0) == 0x90) { t.type = TT_ARRAY; t.len = b & 0x0f; t.total = 1; return true; }
  if ((b & 0xe0) == 0xa0) { t.type = TT_STRING; t.len = b & 0x1f; t.total = 1 + t.len; return t.total <= n; }
  uint32_t need;
  switch (b) {
    case 0xc0: t.type = TT_NIL; t.total = 1; return true;
    case 0xc2: case 0xc3: t.type = TT_BOOLEAN; t.bval = b == 0xc3; t.total = 1; return true;
    case 0xcc: if (n < 2) return false; t.type = TT_INTEGER; t.ival = p[1]; t.total = 2; return true;
    case 0xcd: if (n < 3) return false; t.type = TT_INTEGER; t.ival = be16(p + 1); t.total = 3; return true;
    case 0xce: if (n < 5) return false; t.type = TT_INTEGER; t.ival = be32(p + 1); t.total = 5; return true;
    case 0xcf: if (n < 9) return false; t.type = TT_INTEGER; t.ival = (int64_t)be64(p + 1); t.total = 9;
      return t.ival >= 0;  // MsgPackReader.ensurePositive
    case 0xd0: if (n < 2) return false; t.type = TT_INTEGER; t.ival = (int8_t)p[1]; t.total = 2; return true;
    case 0xd1: if (n < 3) return false; t.type = TT_INTEGER; t.ival = (int16_t)be16(p + 1); t.total = 3; return true;
    case 0xd2: if (n < 5) return false; t.type = TT_INTEGER; t.ival = (int32_t)be32(p + 1); t.total = 5; return true;
    case 0xd3: if (n < 9) return false; t.type = TT_INTEGER; t.ival = (int64_t)be64(p + 1); t.total = 9; return true;
    case 0xca: {
      if (n < 5) return false;
      uint32_t u = be32(p + 1);
      t.type = TT_FLOAT; t.fval = (double)__builtin_bit_cast(float, u); t.total = 5; return true;
    }
    case 0xcb: {
      if (n < 9) return false;
      t.type = TT_FLOAT; t.fval = __builtin_bit_cast(double, be64(p + 1)); t.total = 9; return true;
    }
    case 0xd9: if (n < 2) return false; t.type = TT_STRING; t.len = p[1]; t.hdr = 2; break;
    case 0xda: if (n < 3) return false; t.type = TT_STRING; t.len = be16(p + 1); t.hdr = 3; break;
    case 0xdb: if (n < 5) return false; t.type = TT_STRING; t.len = be32(p + 1); t.hdr = 5; break;
    case 0xc4: if (n < 2) return false; t.type = TT_BINARY; t.len = p[1]; t.hdr = 2; break;
    case 0xc5: if (n < 3) return false; t.type = TT_BINARY; t.len = be16(p + 1); t.hdr = 3; break;
    case 0xc6: if (n < 5) return false; t.type = TT_BINARY; t.len = be32(p + 1); t.hdr = 5; break;
    case 0xdc: if (n < 3) return false; t.type = TT_ARRAY; t.len = be16(p + 1); t.total = 3; return true;
    case 0xdd: if (n < 5) return false; t.type = TT_ARRAY; t.len = be32(p + 1); t.total = 5; return true;
    case 0xde: if (n < 3) return false; t.type = TT_MAP; t.len = be16(p + 1); t.total = 3; return true;
    case 0xdf: if (n < 5) return false; t.type = TT_MAP; t.len = be32(p + 1); t.total = 5; return true;
    default: return false;  // extensions / never-used: "Unsupported token format"
  }
  need = t.hdr + t.len;
  if (need > n || (int32_t)t.len < 0) return false;
  t.total = need;
  return true;
}

// Returns the offset just past the value starting at pos, or 0xffffffff if malformed.
ZB_HD inline uint32_t skip_value(const uint8_t* d, uint32_t n, uint32_t pos) {
  uint64_t pending = 1;
  while (pending > 0) {
    Tok t;
    if (pos >= n || !read_tok(d + pos, n - pos, t)) return 0xffffffffu;
    pos += t.total;
    pending -= 1;
    if (t.type == TT_MAP) pending += 2ull * t.len;
    else if (t.type == TT_ARRAY) pending += t.len;
  }
  return pos;
}

ZB_HD __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

// ------------------------------------------------------------------------------ json-path
struct QueryResult {
  uint32_t count;   // number of results (saturating)
  uint32_t pos, len;  // first result
};

// [ROOT, MAP_KEY k] fast path: every top-level value under key k (the executor's results for this
// two-filter query are exactly those, in document order; container values are whole results).
ZB_HD inline bool query_fast(const uint8_t* d, uint32_t n, const uint8_t* key, uint32_t klen,
                                  QueryResult& r) {
  r.count = 0; r.pos = 0; r.len = 0;
  Tok t;
  if (!read_tok(d, n, t)) return n == 0;
  if (t.type != TT_MAP) return true;  // root filter needs a container; arrays give no key matches
  uint32_t pos = t.total;
  for (uint32_t i = 0; i < t.len; i++) {
    Tok k;
    if (pos >= n || !read_tok(d + pos, n - pos, k)) return false;
    uint32_t kpos = pos;
    pos += k.total;
    uint32_t vend = skip_value(d, n, pos);
    if (vend == 0xffffffffu) return false;
    if (k.type == TT_STRING && k.len == klen && bytes_eq(d + kpos + k.hdr, key, klen)) {
      if (r.count == 0) { r.pos = pos; r.len = vend - pos; }
      r.count++;
    } else if (k.type == TT_MAP || k.type == TT_ARRAY) {
      return false;  // container map keys: the reference's traversal would descend; not supported here
    }
    pos = vend;
  }
  return true;
}

// General executor (literal state machine of MsgPackQueryExecutor.visitElement), depth <= 30.
constexpr int JP_MAX_DEPTH = 30;
// (the traversal state per open container lives in caller-provided arrays of maxd entries)
ZB_HD __forceinline__ bool query_walk(const uint8_t* d, uint32_t n, const DevFilter* f, uint32_t nf,
                                     const uint8_t* pool, QueryResult& r, int* cur, int* num, int* app, int* dyn,
                                     bool* ismap, int maxd) {
  r.count = 0; r.pos = 0; r.len = 0;
  int depth = 0;
  int matching = -1;
  uint32_t mstart = 0;
  uint32_t pos = 0;
  if (nf == 0) return true;
  while (pos < n) {
    Tok t;
    if (!read_tok(d + pos, n - pos, t)) return true;  // traverser stops on an invalid token
    int cf = 0;
    if (depth > 0) { cur[depth - 1] += 1; cf = app[depth - 1]; }
    bool match = false;
    if (cf >= 0) {
      const DevFilter& F = f[cf];
      switch (F.id) {
        case F_ROOT: match = depth == 0 && (t.type == TT_MAP || t.type == TT_ARRAY); break;
        case F_MAP_KEY:
          if (depth > 0 && ismap[depth - 1]) {
            int L = depth - 1;
            if (cur[L] == 0) dyn[L] = -1;
            if (cur[L] == dyn[L]) { dyn[L] = -1; match = true; }
            else if (cur[L] % 2 == 0 && t.type == TT_STRING && t.len == F.key_len &&
                     bytes_eq(d + pos + t.hdr, pool + F.key_off, F.key_len))
              dyn[L] = cur[L] + 1;
          }
          break;
        case F_INDEX: match = depth > 0 && !ismap[depth - 1] && F.index == cur[depth - 1]; break;
        case F_WILDCARD: match = (depth > 0 && ismap[depth - 1]) ? (cur[depth - 1] % 2 != 0) : true; break;
      }
    }
    if (t.type == TT_MAP || t.type == TT_ARRAY) {
      if (depth >= maxd) return false;
      cur[depth] = -1;
      num[depth] = t.type == TT_MAP ? 2 * (int)t.len : (int)t.len;
      app[depth] = -1;
      ismap[depth] = t.type == TT_MAP;
      dyn[depth] = 0;
      depth++;
    }
    if (match) {
      if ((uint32_t)cf + 1 == nf) {
        if (t.type != TT_MAP && t.type != TT_ARRAY) {
          if (r.count == 0) { r.pos = pos; r.len = t.total; }
          r.count++;
        } else {
          matching = depth - 1;
          mstart = pos;
        }
      } else {
        app[depth - 1 < 0 ? 0 : depth - 1] = cf + 1;
      }
    }
    pos += t.total;
    while (depth > 0 && cur[depth - 1] + 1 >= num[depth - 1]) {
      if (matching == depth - 1) {
        if (r.count == 0) { r.pos = mstart; r.len = pos - mstart; }
        r.count++;
        matching = -1;
      }
      depth--;
    }
  }
  return true;
}

ZB_HD inline __noinline__ bool query_general(const uint8_t* d, uint32_t n, const DevFilter* f, uint32_t nf,
                                            const uint8_t* pool, QueryResult& r) {
  int cur[JP_MAX_DEPTH], num[JP_MAX_DEPTH], app[JP_MAX_DEPTH], dyn[JP_MAX_DEPTH];
  bool ismap[JP_MAX_DEPTH];
  return query_walk(d, n, f, nf, pool, r, cur, num, app, dyn, ismap, JP_MAX_DEPTH);
}

ZB_HD inline bool run_query(const uint8_t* d, uint32_t n, const DevQuery& q, const DevFilter* filters,
                                 const uint8_t* pool, QueryResult& r) {
  if (q.fast) {
    const DevFilter& k = filters[q.first + 1];
    return query_fast(d, n, pool + k.key_off, k.key_len, r);
  }
  return query_general(d, n, filters + q.first, q.count, pool, r);
}

// ------------------------------------------------------------------------------ json-el VM
struct CondOut {
  uint8_t err;   // 0 ok, else ErrCode
  uint8_t a, b;  // type codes / args
  uint16_t q;    // query index for path errors
};

struct Operand {
  uint8_t type;
  bool bval;
  int64_t ival;
  double fval;
  const uint8_t* s;
  uint32_t slen;
};

__device__ inline bool load_operand(bool is_path, uint32_t idx, const uint8_t* doc, uint32_t n, const DevConst* consts,
                                    const DevQuery* queries, const DevFilter* filters, const uint8_t* pool,
                                    Operand& o, CondOut& out, bool& unsupported) {
  if (!is_path) {
    const DevConst& c = consts[idx];
    o.type = c.type; o.bval = c.bval; o.ival = c.ival; o.fval = c.fval; o.s = pool + c.str_off; o.slen = c.str_len;
    return true;
  }
  QueryResult r;
  if (!run_query(doc, n, queries[idx], filters, pool, r)) { unsupported = true; return false; }
  if (r.count == 0) { out.err = EC_PATH_NO_RESULT; out.q = (uint16_t)idx; return false; }
  if (r.count > 1) { out.err = EC_PATH_MULTI; out.q = (uint16_t)idx; return false; }
  Tok t;
  if (!read_tok(doc + r.pos, r.len, t)) { unsupported = true; return false; }
  o.type = t.type; o.bval = t.bval; o.ival = t.ival; o.fval = t.fval;
  o.s = doc + r.pos + t.hdr; o.slen = t.len;
  return true;
}

// ensureSameType: INTEGER<->FLOAT promotion, else error on type mismatch
__device__ __forceinline__ bool same_type(Operand& x, Operand& y, CondOut& out) {
  if (x.type == TT_INTEGER && y.type == TT_FLOAT) { x.type = TT_FLOAT; x.fval = (double)x.ival; }
  else if (x.type == TT_FLOAT && y.type == TT_INTEGER) { y.type = TT_FLOAT; y.fval = (double)y.ival; }
  else if (x.type != y.type) { out.err = EC_DIFF_TYPES; out.a = x.type; out.b = y.type; return false; }
  return true;
}

// Evaluates one compiled condition; returns result (valid when out.err == 0 && !unsupported).
// Inlined form: a caller whose document is in LDS gets LDS loads (address-space inference).
template <typename DocPtr>
__device__ __forceinline__ bool eval_condition_inl(uint32_t pc, const uint32_t* code, DocPtr doc, uint32_t n,
                                                   const DevConst* consts, const DevQuery* queries,
                                                   const DevFilter* filters, const uint8_t* pool, CondOut& out,
                                                   bool& unsupported) {
  bool r = false;
  out.err = 0;
  for (int guard = 0; guard < 4096; guard++) {
    uint32_t w0 = code[2 * pc], w1 = code[2 * pc + 1];
    uint32_t opc = w0 & 0xff;
    if (opc == PC_END) return r;
    if (opc == PC_JF) { if (!r) { pc = w0 >> 16; continue; } pc++; continue; }
    if (opc == PC_JT) { if (r) { pc = w0 >> 16; continue; } pc++; continue; }
    // PC_CMP
    uint32_t op = (w0 >> 8) & 0xf;
    Operand x, y;
    if (!load_operand((w0 >> 12) & 1, w1 & 0xffff, doc, n, consts, queries, filters, pool, x, out, unsupported))
      return false;
    if (!load_operand((w0 >> 13) & 1, w1 >> 16, doc, n, consts, queries, filters, pool, y, out, unsupported))
      return false;
    if (op == OP_EQ || op == OP_NE) {
      bool eq;
      if (x.type == TT_NIL) eq = y.type == TT_NIL;
      else if (y.type == TT_NIL) eq = false;
      else {
        if (!same_type(x, y, out)) return false;
        switch (x.type) {
          case TT_STRING: eq = x.slen == y.slen && bytes_eq(x.s, y.s, x.slen); break;
          case TT_BOOLEAN: eq = x.bval == y.bval; break;
          case TT_INTEGER: eq = x.ival == y.ival; break;
          case TT_FLOAT: eq = x.fval == y.fval; break;
          default: out.err = EC_CMP_TYPE; out.a = x.type; return false;
        }
      }
      r = (op == OP_EQ) ? eq : !eq;
    } else {
      if (!same_type(x, y, out)) return false;
      if (x.type != TT_INTEGER && x.type != TT_FLOAT) { out.err = EC_NOT_NUMBER; out.a = x.type; return false; }
      if (x.type == TT_INTEGER) {
        r = op == OP_LT ? x.ival < y.ival : op == OP_LE ? x.ival <= y.ival : op == OP_GT ? x.ival > y.ival
                                                                                       : x.ival >= y.ival;
      } else {
        r = op == OP_LT ? x.fval < y.fval : op == OP_LE ? x.fval <= y.fval : op == OP_GT ? x.fval > y.fval
                                                                                       : x.fval >= y.fval;
      }
    }
    pc++;
  }
  unsupported = true;
  return false;
}
__device__ __noinline__ bool eval_condition(uint32_t pc, const uint32_t* code, const uint8_t* doc, uint32_t n,
                                            const DevConst* consts, const DevQuery* queries, const DevFilter* filters,
                                            const uint8_t* pool, CondOut& out, bool& unsupported) {
  return eval_condition_inl(pc, code, doc, n, consts, queries, filters, pool, out, unsupported);
}

// ------------------------------------------------------------------------------ merge
// Top-level merge(source = job/message payload, target = scope payload), MappingProcessor.merge
// without mappings. Implemented structurally (write_node below):
//   root children = target keys (document order) then source keys not in target;
//   value = source's if present (MsgPackTree.merge: source node types/leaves win, non-root child
//   sets replaced), else target's; a target *leaf* at the same path as a source container wins
//   (stale leafMap entry; MsgPackDocumentTreeWriter checks isLeaf first).
// Containers are re-encoded with minimal headers and keys re-encoded as minimal strings, leaves
// copied raw (MsgPackDocumentTreeWriter.writeNode). Unsupported (flagged): duplicate keys, keys
// containing '[' / ']' (node-id collisions in the reference), non-string keys, depth > MERGE_MAX_DEPTH.
constexpr int MERGE_MAX_DEPTH = 16;

struct Out {
  uint8_t* dst;   // nullptr: size pass
  uint32_t n;
  ZB_HD __forceinline__ void put(uint8_t b) { if (dst) dst[n] = b; n++; }
  ZB_HD __forceinline__ void put_bytes(const uint8_t* s, uint32_t len) {
    if (dst) for (uint32_t i = 0; i < len; i++) dst[n + i] = s[i];
    n += len;
  }
  ZB_HD inline void map_hdr(uint32_t c) {
    if (c < 16) put(0x80 | c);
    else if (c < 65536) { put(0xde); put(c >> 8); put(c & 0xff); }
    else { put(0xdf); put(c >> 24); put((c >> 16) & 0xff); put((c >> 8) & 0xff); put(c & 0xff); }
  }
  ZB_HD inline void arr_hdr(uint32_t c) {
    if (c < 16) put(0x90 | c);
    else if (c < 65536) { put(0xdc); put(c >> 8); put(c & 0xff); }
    else { put(0xdd); put(c >> 24); put((c >> 16) & 0xff); put((c >> 8) & 0xff); put(c & 0xff); }
  }
  ZB_HD inline void str(const uint8_t* s, uint32_t c) {
    if (c < 32) put(0xa0 | c);
    else if (c < 256) { put(0xd9); put(c); }
    else if (c < 65536) { put(0xda); put(c >> 8); put(c & 0xff); }
    else { put(0xdb); put(c >> 24); put((c >> 16) & 0xff); put((c >> 8) & 0xff); put(c & 0xff); }
    put_bytes(s, c);
  }
};

// Out with a capacity: bytes at or past cap are counted but not written (the exact tree's single write pass into a
// preallocated blob: an oversized result is detected by n > cap with nothing written past the blob)
struct OutCap {
  uint8_t* dst;
  uint32_t n;
  uint32_t cap;
  ZB_HD __forceinline__ void put(uint8_t b) { if (n < cap) dst[n] = b; n++; }
  ZB_HD __forceinline__ void put_bytes(const uint8_t* s, uint32_t len) {
    const uint32_t k = n < cap ? (cap - n < len ? cap - n : len) : 0u;
    for (uint32_t i = 0; i < k; i++) dst[n + i] = s[i];
    n += len;
  }
  ZB_HD inline void map_hdr(uint32_t c) {
    if (c < 16) put(0x80 | c);
    else if (c < 65536) { put(0xde); put(c >> 8); put(c & 0xff); }
    else { put(0xdf); put(c >> 24); put((c >> 16) & 0xff); put((c >> 8) & 0xff); put(c & 0xff); }
  }
  ZB_HD inline void arr_hdr(uint32_t c) {
    if (c < 16) put(0x90 | c);
    else if (c < 65536) { put(0xdc); put(c >> 8); put(c & 0xff); }
    else { put(0xdd); put(c >> 24); put((c >> 16) & 0xff); put((c >> 8) & 0xff); put(c & 0xff); }
  }
  ZB_HD inline void str(const uint8_t* s, uint32_t c) {
    if (c < 32) put(0xa0 | c);
    else if (c < 256) { put(0xd9); put(c); }
    else if (c < 65536) { put(0xda); put(c >> 8); put(c & 0xff); }
    else { put(0xdb); put(c >> 24); put((c >> 16) & 0xff); put((c >> 8) & 0xff); put(c & 0xff); }
    put_bytes(s, c);
  }
};

__device__ inline bool key_ok(const uint8_t* s, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (s[i] == '[' || s[i] == ']') return false;
  return true;
}

// Is the key (bytes) the canonical decimal form of an array index? (node ids "$[a][0]" collide for
// map key "0" and array element 0, MsgPackTreeNodeIdConstructor.construct)
__device__ inline bool parse_index(const uint8_t* s, uint32_t n, uint32_t& idx) {
  if (n == 0 || n > 9) return false;
  if (n > 1 && s[0] == '0') return false;
  uint32_t v = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
  }
  idx = v;
  return true;
}

constexpr uint32_t NONE_POS = 0xffffffffu;

// child of the container at cpos (in doc d) named by a map key (kp,kn) or an array index (when kp == nullptr).
// Returns NONE_POS when absent; sets unsupported on duplicate keys.
__device__ inline uint32_t child_of(const uint8_t* d, uint32_t n, uint32_t cpos, const uint8_t* kp, uint32_t kn,
                                    uint32_t index, bool& unsupported) {
  if (cpos == NONE_POS) return NONE_POS;
  Tok c;
  if (!read_tok(d + cpos, n - cpos, c)) return NONE_POS;
  uint32_t pos = cpos + c.total;
  if (c.type == TT_ARRAY) {
    uint32_t want = index;
    if (kp && !parse_index(kp, kn, want)) return NONE_POS;
    if (want >= c.len) return NONE_POS;
    for (uint32_t i = 0; i < want; i++) {
      pos = skip_value(d, n, pos);
      if (pos == 0xffffffffu) return NONE_POS;
    }
    return pos;
  }
  // map: match the key text (array index -> its decimal text)
  uint8_t buf[10];
  if (!kp) {
    uint32_t v = index, l = 0;
    uint8_t tmp[10];
    do { tmp[l++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
    for (uint32_t i = 0; i < l; i++) buf[i] = tmp[l - 1 - i];
    kp = buf;
    kn = l;
  }
  uint32_t found = NONE_POS;
  for (uint32_t i = 0; i < c.len; i++) {
    Tok k;
    if (pos >= n || !read_tok(d + pos, n - pos, k)) return NONE_POS;
    uint32_t vp = pos + k.total;
    if (k.type == TT_STRING && k.len == kn && bytes_eq(d + pos + k.hdr, kp, kn)) {
      if (found != NONE_POS) { unsupported = true; return NONE_POS; }
      found = vp;
    }
    pos = skip_value(d, n, vp);
    if (pos == 0xffffffffu) return NONE_POS;
  }
  return found;
}

// Writes the node at spos of document `d` as MsgPackDocumentTreeWriter would when the other
// document `t` holds the node tpos at the same path (NONE_POS: no node there): a leaf of `t`
// shadows a container of `d` (stale leafMap entry wins isLeaf); otherwise `d`'s structure is
// written with minimal headers / re-encoded keys and its leaves copied raw.
// Returns false when malformed (unsupported set separately).
__device__ __noinline__ bool write_node(const uint8_t* d, uint32_t n, uint32_t spos, const uint8_t* t, uint32_t tn,
                                  uint32_t tpos, Out& o, bool& unsupported) {
  struct Frame {
    uint32_t next, remaining, tcont, idx;
    bool is_map;
  };
  Frame st[MERGE_MAX_DEPTH];
  int depth = 0;
  uint32_t cur_s = spos, cur_t = tpos;
  for (;;) {
    // ---- handle node (cur_s, cur_t)
    Tok ts;
    if (cur_s >= n || !read_tok(d + cur_s, n - cur_s, ts)) return false;
    const bool s_cont = ts.type == TT_MAP || ts.type == TT_ARRAY;
    bool t_leaf = false, t_cont = false;
    Tok tt;
    if (cur_t != NONE_POS) {
      if (!read_tok(t + cur_t, tn - cur_t, tt)) return false;
      t_cont = tt.type == TT_MAP || tt.type == TT_ARRAY;
      t_leaf = !t_cont;
    }
    if (!s_cont) {
      o.put_bytes(d + cur_s, ts.total);
    } else if (t_leaf) {
      o.put_bytes(t + cur_t, tt.total);
    } else {
      if (ts.type == TT_MAP) {
        // keys must be unique strings without brackets (LinkedHashSet dedup / node-id collisions)
        uint32_t kp = cur_s + ts.total;
        for (uint32_t i = 0; i < ts.len; i++) {
          Tok ki;
          if (kp >= n || !read_tok(d + kp, n - kp, ki)) return false;
          if (ki.type != TT_STRING || !key_ok(d + kp + ki.hdr, ki.len)) { unsupported = true; return true; }
          uint32_t vend_i = skip_value(d, n, kp + ki.total);
          if (vend_i == 0xffffffffu) return false;
          uint32_t kj = vend_i;
          for (uint32_t j = i + 1; j < ts.len; j++) {
            Tok kk;
            if (kj >= n || !read_tok(d + kj, n - kj, kk)) return false;
            if (kk.type == TT_STRING && kk.len == ki.len && bytes_eq(d + kj + kk.hdr, d + kp + ki.hdr, ki.len)) {
              unsupported = true;
              return true;
            }
            kj = skip_value(d, n, kj + kk.total);
            if (kj == 0xffffffffu) return false;
          }
          kp = vend_i;
        }
        o.map_hdr(ts.len);
      } else {
        o.arr_hdr(ts.len);
      }
      if (ts.len > 0) {
        if (depth >= MERGE_MAX_DEPTH) { unsupported = true; return true; }
        st[depth++] = Frame{cur_s + ts.total, ts.len, t_cont ? cur_t : NONE_POS, 0, ts.type == TT_MAP};
      }
    }
    // ---- next child
    for (;;) {
      if (depth == 0) return true;
      Frame& f = st[depth - 1];
      if (f.remaining == 0) { depth--; continue; }
      uint32_t vpos;
      if (f.is_map) {
        Tok k;
        if (f.next >= n || !read_tok(d + f.next, n - f.next, k)) return false;
        o.str(d + f.next + k.hdr, k.len);
        vpos = f.next + k.total;
        cur_t = child_of(t, tn, f.tcont, d + f.next + k.hdr, k.len, 0, unsupported);
      } else {
        vpos = f.next;
        cur_t = child_of(t, tn, f.tcont, nullptr, 0, f.idx, unsupported);
      }
      if (unsupported) return true;
      uint32_t vend = skip_value(d, n, vpos);
      if (vend == 0xffffffffu) return false;
      f.next = vend;
      f.remaining--;
      f.idx++;
      cur_s = vpos;
      break;
    }
  }
}

struct RootEntry {
  uint32_t kpos, klen, vpos, vend;
};

// find key in a root map starting after the header; returns entry via e (vpos==0 if absent)
__device__ inline bool find_key(const uint8_t* d, uint32_t n, uint32_t first, uint32_t count, const uint8_t* key,
                                uint32_t klen, RootEntry& e) {
  uint32_t pos = first;
  for (uint32_t i = 0; i < count; i++) {
    Tok k;
    if (pos >= n || !read_tok(d + pos, n - pos, k)) return false;
    uint32_t vp = pos + k.total;
    uint32_t ve = skip_value(d, n, vp);
    if (ve == 0xffffffffu) return false;
    if (k.type == TT_STRING && k.len == klen && bytes_eq(d + pos + k.hdr, key, klen)) {
      e.kpos = pos + k.hdr; e.klen = k.len; e.vpos = vp; e.vend = ve;
      return true;
    }
    pos = ve;
  }
  e.vpos = 0;
  return true;
}

// Validates a root map: string keys, no brackets, no duplicates. Returns false on malformed.
__device__ inline bool check_root(const uint8_t* d, uint32_t n, uint32_t first, uint32_t count, bool& unsupported) {
  uint32_t pos = first;
  for (uint32_t i = 0; i < count; i++) {
    Tok k;
    if (pos >= n || !read_tok(d + pos, n - pos, k)) return false;
    if (k.type != TT_STRING || !key_ok(d + pos + k.hdr, k.len)) { unsupported = true; return true; }
    uint32_t vp = pos + k.total;
    uint32_t ve = skip_value(d, n, vp);
    if (ve == 0xffffffffu) return false;
    // duplicates among later keys
    RootEntry e;
    uint32_t rest = ve;
    uint32_t remaining = count - i - 1;
    if (remaining > 0) {
      if (!find_key(d, n, rest, remaining, d + pos + k.hdr, k.len, e)) return false;
      if (e.vpos != 0) { unsupported = true; return true; }
    }
    pos = ve;
  }
  return true;
}

// Every map key in the document is a string, as MsgPackDocumentIndexer requires of both documents it indexes (it
// throws on any other key, anywhere -- also under a container the merge later shadows). False also for documents
// nested deeper than the check's stack and for unreadable tokens: the exact tree (zb_xmerge.hpp) takes those.
ZB_HD inline bool keys_are_strings(const uint8_t* d, uint32_t n) {
  constexpr int D = 32;
  uint32_t rem[D];
  bool is_map[D];
  int depth = 0;
  uint32_t pos = 0;
  bool root = true;
  while (root || depth > 0) {
    if (depth > 0 && rem[depth - 1] == 0) { depth--; continue; }
    Tok t;
    if (pos >= n || !read_tok(d + pos, n - pos, t)) return false;
    if (depth > 0) {
      const uint32_t k = --rem[depth - 1];
      if (is_map[depth - 1] && (k & 1) && t.type != TT_STRING) return false;  // an odd count left: a key
    }
    root = false;
    pos += t.total;
    if (t.type == TT_MAP || t.type == TT_ARRAY) {
      if (depth == D) return false;
      rem[depth] = t.type == TT_MAP ? 2 * t.len : t.len;
      is_map[depth] = t.type == TT_MAP;
      depth++;
    }
  }
  return true;
}

// Performs the merge into o (size pass when o.dst == nullptr). Returns false when malformed -- and for any
// document keys_are_strings refuses: the exact tree gives the reference's outcome for those.
__device__ __noinline__ bool merge_docs(const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt, Out& o,
                                  bool& unsupported) {
  Tok ts, tt;
  bool src_nil = ns == 0 || (ns >= 1 && src[0] == 0xc0);
  bool tgt_nil = nt == 0 || (nt >= 1 && tgt[0] == 0xc0);
  if (!src_nil && (!read_tok(src, ns, ts) || ts.type != TT_MAP)) { unsupported = true; return true; }
  if (!tgt_nil && (!read_tok(tgt, nt, tt) || tt.type != TT_MAP)) { unsupported = true; return true; }
  // empty tree -> writeNil; the only consumer (DocumentValue.wrap) turns NIL into {} (0x80)
  if (src_nil && tgt_nil) { o.put(0x80); return true; }
  uint32_t sc = src_nil ? 0 : ts.len, tc = tgt_nil ? 0 : tt.len;
  uint32_t sf = src_nil ? 0 : ts.total, tf = tgt_nil ? 0 : tt.total;
  if ((!src_nil && !keys_are_strings(src, ns)) || (!tgt_nil && !keys_are_strings(tgt, nt))) return false;
  if (!src_nil && !check_root(src, ns, sf, sc, unsupported)) return false;
  if (!tgt_nil && !check_root(tgt, nt, tf, tc, unsupported)) return false;
  if (unsupported) return true;
  // count result keys
  uint32_t total = tc;
  {
    uint32_t pos = sf;
    for (uint32_t i = 0; i < sc; i++) {
      Tok k;
      read_tok(src + pos, ns - pos, k);
      RootEntry e;
      if (!find_key(tgt, nt, tf, tc, src + pos + k.hdr, k.len, e)) return false;
      if (e.vpos == 0) total++;
      pos = skip_value(src, ns, pos + k.total);
    }
  }
  o.map_hdr(total);
  // target keys in order
  uint32_t pos = tf;
  for (uint32_t i = 0; i < tc; i++) {
    Tok k;
    read_tok(tgt + pos, nt - pos, k);
    uint32_t vp = pos + k.total;
    uint32_t ve = skip_value(tgt, nt, vp);
    o.str(tgt + pos + k.hdr, k.len);
    RootEntry e;
    if (!find_key(src, ns, sf, sc, tgt + pos + k.hdr, k.len, e)) return false;
    if (e.vpos == 0) {
      if (!write_node(tgt, nt, vp, nullptr, 0, NONE_POS, o, unsupported)) return false;  // target only
    } else {
      // source node wins, except where the target holds a leaf at the same path
      if (!write_node(src, ns, e.vpos, tgt, nt, vp, o, unsupported)) return false;
    }
    if (unsupported) return true;
    pos = ve;
  }
  // source keys not in target
  pos = sf;
  for (uint32_t i = 0; i < sc; i++) {
    Tok k;
    read_tok(src + pos, ns - pos, k);
    uint32_t vp = pos + k.total;
    RootEntry e;
    if (!find_key(tgt, nt, tf, tc, src + pos + k.hdr, k.len, e)) return false;
    uint32_t ve;
    ve = skip_value(src, ns, vp);
    if (ve == 0xffffffffu) return false;
    if (e.vpos == 0) {
      o.str(src + pos + k.hdr, k.len);
      if (!write_node(src, ns, vp, nullptr, 0, NONE_POS, o, unsupported)) return false;  // source only
      if (unsupported) return true;
    }
    pos = ve;
  }
  return true;
}

// ------------------------------------------------------------------------------ flat merge
// Fast path of merge_docs for the common payload shape: both documents are fixmaps, every key a
// fixstr without '[' / ']', every value a scalar (nil, bool, int, float, fixstr / str8, bin8), no
// duplicate keys. For such documents MappingProcessor.merge reduces to: target keys in document
// order, each with the source value when the source has that key, then the source keys the
// target lacks; leaves are copied raw and fixstr keys are already minimal
// (MsgPackDocumentTreeWriter.writeNode), so the output is exactly merge_docs'. Anything else returns
// false and the caller runs merge_docs. Written as rolled loops that re-parse entries on the fly:
// no per-entry tables, so it stays small in code and registers. The byte accesses go through plain
// pointers, so the kernels point them at LDS copies of the documents (zb_traj.hip).

// length of the scalar value at d[p] (n bytes in the document), 0 = not a supported scalar
__device__ __forceinline__ uint32_t flat_scalar_len(const uint8_t* d, uint32_t n, uint32_t p) {
  if (p >= n) return 0;
  const uint32_t b = d[p];
  uint32_t len;
  if (b <= 0x7f || b >= 0xe0 || b == 0xc0 || b == 0xc2 || b == 0xc3) len = 1;
  else if ((b & 0xe0) == 0xa0) len = 1 + (b & 0x1f);
  else if (b == 0xcc || b == 0xd0) len = 2;
  else if (b == 0xcd || b == 0xd1) len = 3;
  else if (b == 0xce || b == 0xd2 || b == 0xca) len = 5;
  else if (b == 0xd3 || b == 0xcb) len = 9;  // 0xcf (uint64) needs the ensurePositive check: general path
  else if (b == 0xd9 || b == 0xc4) { if (p + 1 >= n) return 0; len = 2 + d[p + 1]; }
  else return 0;
  return p + len <= n ? len : 0;
}

// entry at p: fixstr key of kl bytes at p + 1, scalar value of vl bytes at p + 1 + kl
__device__ __forceinline__ bool flat_entry(const uint8_t* d, uint32_t n, uint32_t p, uint32_t& kl, uint32_t& vl) {
  if (p >= n) return false;
  const uint32_t kb = d[p];
  if ((kb & 0xe0) != 0xa0) return false;
  kl = kb & 0x1f;
  if (p + 1 + kl > n) return false;
  vl = flat_scalar_len(d, n, p + 1 + kl);
  return vl != 0;
}

__device__ __forceinline__ bool flat_bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t j = 0; j < n; j++)
    if (a[j] != b[j]) return false;
  return true;
}

// Value (position | length << 16) of key k in the flat map d with cnt entries; 0 when absent.
__device__ __forceinline__ uint32_t flat_find(const uint8_t* d, uint32_t n, uint32_t cnt, const uint8_t* k,
                                              uint32_t klen) {
  uint32_t p = 1, found = 0;
  for (uint32_t i = 0; i < cnt; i++) {
    uint32_t kl, vl;
    flat_entry(d, n, p, kl, vl);
    if (!found && kl == klen && flat_bytes_eq(d + p + 1, k, kl)) found = (p + 1 + kl) | (vl << 16);
    p += 1 + kl + vl;
  }
  return found;
}

// Checks the document is a flat map (or nil: cnt = 0) without duplicate or '['/']' keys.
__device__ __forceinline__ bool flat_check(const uint8_t* d, uint32_t n, uint32_t& cnt) {
  cnt = 0;
  if (n == 0 || (n == 1 && d[0] == 0xc0)) return true;  // nil document = empty tree
  const uint32_t h = d[0];
  if ((h & 0xf0) != 0x80 || n > 0xffff) return false;
  cnt = h & 0x0f;
  uint32_t p = 1;
  for (uint32_t i = 0; i < cnt; i++) {
    uint32_t kl, vl;
    if (!flat_entry(d, n, p, kl, vl)) return false;
    for (uint32_t j = 0; j < kl; j++) {
      const uint8_t c = d[p + 1 + j];
      if (c == '[' || c == ']') return false;
    }
    // duplicates among the later entries (merge_docs flags them unsupported)
    uint32_t q = p + 1 + kl + vl;
    for (uint32_t j = i + 1; j < cnt; j++) {
      uint32_t kl2, vl2;
      if (!flat_entry(d, n, q, kl2, vl2)) return false;
      if (kl2 == kl && flat_bytes_eq(d + q + 1, d + p + 1, kl)) return false;
      q += 1 + kl2 + vl2;
    }
    p += 1 + kl + vl;
  }
  return p == n;
}

// Writes merge(src -> tgt) to out (capacity cap) and its length to olen; false = not flat.
__device__ __forceinline__ bool merge_flat(const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt,
                                           uint8_t* out, uint32_t cap, uint32_t& olen) {
  uint32_t sc, tc;
  if (ns + nt + 3 > cap || !flat_check(src, ns, sc) || !flat_check(tgt, nt, tc)) return false;
  // result keys: the target's, then the source's the target lacks
  uint32_t total = tc, p = 1;
  for (uint32_t i = 0; i < sc; i++) {
    uint32_t kl, vl;
    flat_entry(src, ns, p, kl, vl);
    if (!flat_find(tgt, nt, tc, src + p + 1, kl)) total++;
    p += 1 + kl + vl;
  }
  // (an empty result is the fixmap header alone, 0x80, as merge_docs writes for an empty tree)
  uint32_t o = 0;
  if (total < 16) out[o++] = (uint8_t)(0x80 | total);
  else { out[o++] = 0xde; out[o++] = 0; out[o++] = (uint8_t)total; }
  p = 1;
  for (uint32_t i = 0; i < tc; i++) {
    uint32_t kl, vl;
    flat_entry(tgt, nt, p, kl, vl);
    for (uint32_t j = 0; j < 1 + kl; j++) out[o++] = tgt[p + j];
    const uint32_t f = flat_find(src, ns, sc, tgt + p + 1, kl);  // the source value wins
    const uint8_t* v = f ? src + (f & 0xffff) : tgt + p + 1 + kl;
    const uint32_t len = f ? (f >> 16) : vl;
    for (uint32_t j = 0; j < len; j++) out[o++] = v[j];
    p += 1 + kl + vl;
  }
  p = 1;
  for (uint32_t i = 0; i < sc; i++) {
    uint32_t kl, vl;
    flat_entry(src, ns, p, kl, vl);
    if (!flat_find(tgt, nt, tc, src + p + 1, kl))
      for (uint32_t j = 0; j < 1 + kl + vl; j++) out[o++] = src[p + j];
    p += 1 + kl + vl;
  }
  olen = o;
  return true;
}

// ------------------------------------------------------------------------------ explicit io-mappings
// MappingProcessor.extract / merge with mappings (json-path/.../mapping/MappingProcessor.java:143-190): the
// target document is indexed into a MsgPackTree (MsgPackDocumentIndexer.java:136-283), every mapping puts its
// source query's single result at its target path (MsgPackDocumentExtractor.java:121-230: createParentRelation,
// executeLeafMapping), and the tree is written out (MsgPackDocumentTreeWriter.java:53-104). The tree lives in a
// caller-provided workspace as nodes identified by (parent, name) -- what the reference's string node ids
// "$[a][b]" identify -- with names taken from the target document's keys, the target path literals (pool) or
// array indices. MsgPackTree keeps node types and leaves apart from the child sets, so a node can carry a leaf
// and a type at once (addArrayNode keeps a leaf, addMapNode drops it); the writer looks at the leaf first.
// Names holding '[' or ']' (where the reference's string ids collide) are flagged unsupported.
constexpr uint32_t MAP_NODES = 256;
constexpr int MAP_DEPTH = 32;
constexpr uint16_t MN_NONE = 0xffff;
enum : uint8_t { MN_UNTYPED = 0, MN_LEAF_T = 1, MN_LEAF_S = 2, MN_MAP = 3, MN_ARRAY = 4 };
enum : uint8_t { NS_TDOC = 0, NS_POOL = 1, NS_INDEX = 2 };
// outcome of map_documents
enum : int { MAP_OK = 0, MAP_ERR_NO_DATA = 1, MAP_ERR_NOT_MAP = 2, MAP_FAIL = 3, MAP_UNSUPPORTED = 4,
             MAP_DONE = 5 /* (k_map: the exact tree wrote the result) */ };

struct MNode {
  uint32_t name;        // name bytes offset (NS_TDOC: target document, NS_POOL: pool) or array index (NS_INDEX)
  uint16_t nlen;
  uint8_t nsrc, type;
  uint32_t lpos, llen;  // leaf value in the target (MN_LEAF_T) or source document; llen 0 = no leaf
  uint16_t first, last, next, pad;
};
static_assert(sizeof(MNode) == 24, "MNode is 24 bytes");

__device__ __forceinline__ bool has_bracket(const uint8_t* p, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (p[i] == '[' || p[i] == ']') return true;
  return false;
}

struct MapTree {
  MNode* n;
  uint32_t cnt;
  const uint8_t* t;  // indexed (target) document
  uint32_t tn;
  const uint8_t* s;  // extract (source) document
  uint32_t sn;
  const uint8_t* pool;
  int status;

  __device__ const uint8_t* name_of(uint8_t src, uint32_t off, uint32_t len, uint8_t* tmp, uint32_t& l) const {
    if (src == NS_TDOC) { l = len; return t + off; }
    if (src == NS_POOL) { l = len; return pool + off; }
    uint8_t d[10];
    int k = 0;
    uint32_t v = off;
    do { d[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
    for (int i = 0; i < k; i++) tmp[i] = d[k - 1 - i];
    l = (uint32_t)k;
    return tmp;
  }
  __device__ uint16_t add_node(uint8_t src, uint32_t off, uint32_t len) {
    if (cnt >= MAP_NODES || len > 0xffff) { status = MAP_UNSUPPORTED; return MN_NONE; }
    MNode& m = n[cnt];
    m.name = off; m.nlen = (uint16_t)len; m.nsrc = src; m.type = MN_UNTYPED; m.lpos = 0; m.llen = 0;
    m.first = m.last = m.next = MN_NONE; m.pad = 0;
    return (uint16_t)cnt++;
  }
  // MsgPackTree.addChildToNode: the parent's child set keeps insertion order and no duplicates
  __device__ uint16_t child(uint16_t parent, uint8_t src, uint32_t off, uint32_t len) {
    uint8_t ta[12], tb[12];
    uint32_t la, lb;
    const uint8_t* a = name_of(src, off, len, ta, la);
    for (uint16_t c = n[parent].first; c != MN_NONE; c = n[c].next) {
      const uint8_t* b = name_of(n[c].nsrc, n[c].name, n[c].nlen, tb, lb);
      if (la == lb && bytes_eq(a, b, la)) return c;
    }
    const uint16_t c = add_node(src, off, len);
    if (c == MN_NONE) return c;
    if (n[parent].last == MN_NONE) n[parent].first = c;
    else n[n[parent].last].next = c;
    n[parent].last = c;
    return c;
  }
  __device__ void add_map(uint16_t x) { n[x].llen = 0; n[x].type = MN_MAP; }    // addMapNode: leaf removed
  __device__ void add_array(uint16_t x) { n[x].type = MN_ARRAY; }               // addArrayNode: leaf kept
  __device__ void add_leaf(uint16_t x, uint32_t pos, uint32_t len, bool extracted) {
    n[x].lpos = pos; n[x].llen = len; n[x].type = extracted ? MN_LEAF_S : MN_LEAF_T;
  }
};

// MsgPackDocumentIndexer.index of the target document into the tree (root node 0)
__device__ inline void map_index(MapTree& T) {
  Tok t;
  if (T.tn == 0 || !read_tok(T.t, T.tn, t) || t.type == TT_NIL) return;  // empty tree
  if (t.type != TT_MAP) { T.status = MAP_UNSUPPORTED; return; }
  uint16_t fnode[MAP_DEPTH];
  uint32_t frem[MAP_DEPTH], fidx[MAP_DEPTH];
  bool farr[MAP_DEPTH];
  int depth = 0;
  T.add_map(0);
  fnode[0] = 0; frem[0] = t.len; fidx[0] = 0; farr[0] = false;
  depth = 1;
  uint32_t pos = t.total;
  while (depth > 0) {
    const int L = depth - 1;
    if (frem[L] == 0) { depth--; continue; }
    frem[L]--;
    uint16_t c;
    if (!farr[L]) {
      Tok k;
      if (pos >= T.tn || !read_tok(T.t + pos, T.tn - pos, k)) { T.status = MAP_UNSUPPORTED; return; }
      if (k.type != TT_STRING) { T.status = MAP_FAIL; return; }  // "non-string map key is not supported"
      if (has_bracket(T.t + pos + k.hdr, k.len)) { T.status = MAP_UNSUPPORTED; return; }
      c = T.child(fnode[L], NS_TDOC, pos + k.hdr, k.len);
      pos += k.total;
    } else {
      c = T.child(fnode[L], NS_INDEX, fidx[L]++, 0);
    }
    if (c == MN_NONE) return;
    Tok v;
    if (pos >= T.tn || !read_tok(T.t + pos, T.tn - pos, v)) { T.status = MAP_UNSUPPORTED; return; }
    if (v.type == TT_MAP || v.type == TT_ARRAY) {
      if (v.type == TT_MAP) T.add_map(c); else T.add_array(c);
      if (depth >= MAP_DEPTH) { T.status = MAP_UNSUPPORTED; return; }
      fnode[depth] = c; frem[depth] = v.len; fidx[depth] = 0; farr[depth] = v.type == TT_ARRAY;
      depth++;
    } else {
      T.add_leaf(c, pos, v.total, false);
    }
    pos += v.total;
  }
}

// MsgPackDocumentExtractor.extract: every mapping's target path, then its source query's result as the leaf
__device__ inline void map_extract(MapTree& T, const DevMapping* maps, uint32_t nmaps, const DevSeg* segs,
                                   const DevQuery* queries, const DevFilter* filters, uint16_t& fail_query) {
  for (uint32_t mi = 0; mi < nmaps; mi++) {
    const DevMapping m = maps[mi];
    uint16_t node = MN_NONE;
    for (uint32_t k = 0; k < m.nseg; k++) {
      const DevSeg sg = segs[m.seg + k];
      const uint8_t* nm = T.pool + sg.off;
      if (has_bracket(nm, sg.len)) { T.status = MAP_UNSUPPORTED; return; }
      if (node == MN_NONE) {  // createParentRelation("", "$") is the root's id
        node = 0;
        continue;
      }
      bool index = true;  // isIndex :168-177 (an empty name counts as an index)
      for (uint32_t i = 0; i < sg.len; i++)
        if (nm[i] < '0' || nm[i] > '9') { index = false; break; }
      if (index) {
        if (T.n[node].type != MN_MAP) T.add_array(node);
      } else {
        T.add_map(node);
      }
      node = T.child(node, NS_POOL, sg.off, sg.len);
      if (node == MN_NONE) return;
    }
    if (node == MN_NONE) { T.status = MAP_UNSUPPORTED; return; }
    QueryResult r;
    if (!run_query(T.s, T.sn, queries[m.query], filters, T.pool, r)) { T.status = MAP_UNSUPPORTED; return; }
    if (r.count == 0) { T.status = MAP_ERR_NO_DATA; fail_query = m.query; return; }
    if (r.count > 1) { T.status = MAP_FAIL; return; }  // IllegalStateException: more than one matching source
    T.add_leaf(node, r.pos, r.len, true);
  }
}

// MsgPackDocumentTreeWriter.write
__device__ inline void map_write(MapTree& T, Out& o) {
  if (T.n[0].type == MN_UNTYPED && T.n[0].llen == 0) { o.put(0xc0); return; }  // empty tree: nil
  uint16_t fnode[MAP_DEPTH + 1];
  bool farr[MAP_DEPTH + 1];
  int depth = 0;
  uint16_t x = 0;
  bool key = false;
  bool arr_parent = false;
  for (;;) {
    // write node x (its key first, unless the parent is an array or x is the root)
    const MNode m = T.n[x];
    if (key && !arr_parent) {
      uint8_t tmp[12];
      uint32_t l;
      const uint8_t* nm = T.name_of(m.nsrc, m.name, m.nlen, tmp, l);
      o.str(nm, l);
    }
    if (m.llen) {
      // the buffer follows the node type, not where the leaf came from (an extracted leaf under a node that
      // addArrayNode retyped is read from the indexed document): out of its bounds the reference's buffer
      // access throws
      const bool from_s = m.type == MN_LEAF_S;
      if ((uint64_t)m.lpos + m.llen > (from_s ? T.sn : T.tn)) { T.status = MAP_FAIL; return; }
      o.put_bytes((from_s ? T.s : T.t) + m.lpos, m.llen);
    } else if (m.type == MN_MAP || m.type == MN_ARRAY) {
      uint32_t nc = 0;
      for (uint16_t c = m.first; c != MN_NONE; c = T.n[c].next) nc++;
      if (m.type == MN_ARRAY) o.arr_hdr(nc); else o.map_hdr(nc);
      if (m.first != MN_NONE) {
        if (depth > MAP_DEPTH) { T.status = MAP_UNSUPPORTED; return; }
        fnode[depth] = m.first;
        farr[depth] = m.type == MN_ARRAY;
        depth++;
        x = m.first; key = true; arr_parent = m.type == MN_ARRAY;
        continue;
      }
    } else {
      T.status = MAP_FAIL;  // a child without node type: NullPointerException in the writer
      return;
    }
    // next sibling, or climb
    for (;;) {
      if (depth == 0) return;
      const uint16_t nx = T.n[fnode[depth - 1]].next;
      if (nx != MN_NONE) {
        fnode[depth - 1] = nx;
        x = nx; key = true; arr_parent = farr[depth - 1];
        break;
      }
      depth--;
    }
  }
}

// The result document of MappingProcessor.extract(src, mappings) (tgt == nullptr) or .merge(src, tgt,
// mappings), nmaps >= 1; the size pass when o.dst == nullptr. Returns MAP_OK, MAP_ERR_NO_DATA (fail_query set)
// or MAP_ERR_NOT_MAP (MappingException -> IO_MAPPING_ERROR incident), MAP_FAIL (any other exception: the
// processor fails) or MAP_UNSUPPORTED. ws: MAP_NODES nodes.
__device__ __noinline__ int map_documents(const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt,
                                          const DevMapping* maps, uint32_t nmaps, const DevSeg* segs,
                                          const DevQuery* queries, const DevFilter* filters, const uint8_t* pool,
                                          MNode* ws, Out& o, uint16_t& fail_query) {
  MapTree T;
  T.n = ws; T.cnt = 0; T.t = tgt; T.tn = tgt ? nt : 0; T.s = src; T.sn = ns; T.pool = pool; T.status = MAP_OK;
  T.add_node(NS_INDEX, 0, 0);  // "$"
  if (tgt) map_index(T);
  if (T.status != MAP_OK) return T.status;
  map_extract(T, maps, nmaps, segs, queries, filters, fail_query);
  if (T.status != MAP_OK) return T.status;
  map_write(T, o);
  if (T.status != MAP_OK) return T.status;
  // ensureDocumentIsAMsgPackMap :206-213: the written document must be a map (or nil)
  const MNode r = T.n[0];
  if (r.llen) {
    const uint8_t b = (r.type == MN_LEAF_S ? src : tgt)[r.lpos];
    if (!((b & 0xf0) == 0x80 || b == 0xde || b == 0xdf || b == 0xc0)) return MAP_ERR_NOT_MAP;
  } else if (r.type == MN_ARRAY) {
    return MAP_ERR_NOT_MAP;
  }
  return MAP_OK;
}

}  // namespace zbg
