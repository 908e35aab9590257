// zb_xmerge.hpp — the exact payload tree of MappingProcessor for the documents the structural merge (merge_docs,
// merge_flat) and the node-table mapper (map_documents) do not take: duplicate keys, keys holding '[' or ']' (where
// the reference's string node ids collide), any nesting depth, any number of nodes up to the workspace.
//
// This is the reference's data structure itself, restated over a flat workspace: nodes are identified by their
// string ids ("$[a][0][b]", MsgPackTreeNodeIdConstructor), looked up by hashing the id bytes, so every collision the
// reference makes between two paths happens here too.
//   MsgPackDocumentIndexer.index / visitElement / addNewParent / processValueNode
//       json-path/src/main/java/io/zeebe/msgpack/mapping/MsgPackDocumentIndexer.java:136-283
//   MsgPackTree add*Node / addChildToNode / merge      json-path/.../mapping/MsgPackTree.java:84-166
//   MsgPackDocumentTreeWriter.write / writeNode        json-path/.../mapping/MsgPackDocumentTreeWriter.java:53-104
//   MsgPackDocumentExtractor.extract / createParentRelation / executeLeafMapping
//       json-path/.../mapping/MsgPackDocumentExtractor.java:121-230
//   MappingProcessor.merge / extract / ensureDocumentIsAMsgPackMap
//       json-path/.../mapping/MappingProcessor.java:143-223
// One thread per document pair over its own slab (XSLAB_BYTES): the kernels that use it (zb_aux.hip, zb_traj.hip)
// take the pairs the fast paths refused, which are rare. Everything here is plain code over the slab, so it also
// builds for the host (tests/xmerge_host.cpp checks it against the oracle over a corpus of odd documents).
#pragma once
#include "zb_devlib.hpp"

namespace zbg {

constexpr uint32_t XSLAB_BYTES = 4u << 20;  // workspace of one document pair
constexpr uint32_t XSLAB_COUNT = 32;        // pairs in flight (zb_xlock.hpp: one lock per slab)
constexpr uint32_t XPOOL_SLACK = 16;        // bytes past a workspace's string pool its 8-byte string chunks may touch
// every lane first tries its pair in a small workspace of its own (XLANE_COUNT of them, held 64 at a time by a wave:
// zb_xlock.hpp x_run): 32 KB holds the tree of ~140 tokens (2 x source + target), the documents of a typical job /
// message payload merge (a larger pair takes the slab path)
constexpr uint32_t XLANE_BYTES = 32u << 10;
constexpr uint32_t XLANE_COUNT = 131072;  // (4 GiB per device, shared by its engines; k_merge_gen's grid: 512 workgroups
                                          //  of 256 lanes. C1 1M exact-tree tick on the trajectory path, one box
                                          //  (profiles/r06/ab_xlanes_r06ac.txt): 64K x 32 KB 3.06 ms, 128K x 32 KB 2.53,
                                          //  128K x 16 KB 2.48 and 256K x 16 KB 2.48 -- but at 16 KB half the pairs of
                                          //  test_xmerge_lane_workspaces_vs_oracle leave for a slab. Before the arrays
                                          //  were interleaved, 64K lanes were best: their scattered lines fell out of
                                          //  the Infinity Cache above that)
constexpr uint32_t XLANE_GROUPS = XLANE_COUNT / 64;          // lane groups (one wave's 64 workspaces)
constexpr uint32_t XLOCK_COUNT = XSLAB_COUNT + XLANE_GROUPS;  // slab locks, then lane-group locks

// node types (MsgPackTree.nodeTypeMap values; XT_NONE = no entry)
enum : uint8_t { XT_NONE = 0, XT_EXISTING_LEAF = 1, XT_EXTRACTED_LEAF = 2, XT_MAP = 3, XT_ARRAY = 4 };
// outcomes: X_FAIL = an exception other than MappingException (the processor fails), X_NO_DATA / X_NOT_MAP = the
// MappingExceptions that become IO_MAPPING_ERROR incidents, X_UNSUP = the workspace or output limit was reached
enum : int { X_OK = 0, X_FAIL = 1, X_NO_DATA = 2, X_NOT_MAP = 3, X_UNSUP = 4 };
constexpr uint32_t XNONE = 0xffffffffu;

struct XStr {  // bytes in the slab's string pool
  uint32_t off, len;
};

// A workspace: bytes per lane at base, shared by S lanes (S = 1: one lane's own slab -- the big slabs, the host). The
// tree's arrays are interleaved element by element over the S lanes (lane l's element j at j * S + l), so the lanes of a
// wave that walk alike -- documents of one shape -- touch adjacent elements, one memory request for many lanes instead
// of one per lane; each lane's string pool is its own contiguous region after the arrays.
struct XWs {
  uint8_t* base;
  uint32_t bytes;  // per lane
  uint32_t lane, S;
};
template <class T>
struct XArr {  // a lane's view of an interleaved array
  T* p;         // its element 0
  uint32_t s;   // stride in elements (S)
  ZB_HD T& operator[](uint32_t j) const { return p[(uint64_t)j * s]; }
};

struct XNode {
  XStr id;
  uint32_t hash;
  uint8_t tree, type, has_leaf, has_childs;  // tree 0: the written tree, 1: the merged-in source tree
  uint32_t lpos, llen;                       // leafMap entry (position / length in the node type's buffer)
  uint32_t cfirst, clast, ccount;            // nodeChildsMap entry: LinkedHashSet<String> as a list of XChild
};

struct XChild {
  XStr name;
  uint32_t next, parent;
};

struct XFrame {  // writer stack: a container being written
  XStr id;
  uint32_t cur;
  uint32_t arr;
};

struct XTree {
  uint8_t* pool;
  uint32_t pool_n, pool_cap;
  XArr<XNode> nodes;
  uint32_t nn, nn_cap;
  XArr<XChild> ch;
  uint32_t nc, nc_cap;
  XArr<uint32_t> ht;  // (tree, id) -> node + 1
  uint32_t ht_mask;
  XArr<uint32_t> hc;  // (parent node, child name) -> child + 1
  uint32_t hc_mask;
  XArr<XStr> st_par;  // the indexer's parentsStack / isArrayValueStack / lastTypeStack (ArrayDeque push/pop at the front)
  XArr<uint8_t> st_arr;
  XArr<uint8_t> st_typ;
  uint32_t n_par, n_arr, n_typ, st_cap;
  XArr<XFrame> fr;
  uint32_t typed[2];  // nodes with a node type, per tree
  XStr dollar;
  int status;

  ZB_HD uint8_t* s(XStr x) const { return pool + x.off; }

  ZB_HD static uint64_t need_of(uint32_t items, uint32_t& n, uint32_t& h) {
    n = items + 16;
    h = 64;
    while (h < 2 * n) h <<= 1;
    return (uint64_t)n * (sizeof(XNode) + sizeof(XChild) + sizeof(XStr) + 2 + sizeof(XFrame)) +
           2ull * h * sizeof(uint32_t) + 64;
  }
  ZB_HD bool init(const XWs& w, uint32_t items) {
    status = X_OK;
    uint32_t n, h;
    if (need_of(items, n, h) > w.bytes / 2) { status = X_UNSUP; return false; }
#ifdef __HIP_DEVICE_COMPILE__
    if (w.S > 1) {
      // the interleaved arrays must have one layout for every lane of the group that uses them at once: the lanes of
      // the wave that got here (each fits) size it for the largest of them
      uint64_t act = __ballot(1);
      uint32_t m = 0;
      while (act) {
        const int l = __ffsll((unsigned long long)act) - 1;
        m = max(m, (uint32_t)__builtin_amdgcn_readlane(items, l));
        act &= act - 1;
      }
      (void)need_of(m, n, h);
    }
#endif
    const uint32_t S = w.S;
    uint64_t off = 0;  // the arrays of all S lanes, then the S pools
    auto take = [&](uint32_t elem, uint64_t count) {
      uint8_t* r = w.base + off + (uint64_t)w.lane * elem;
      off += ((uint64_t)elem * count * S + 15) & ~15ull;
      return r;
    };
    nodes = XArr<XNode>{(XNode*)take(sizeof(XNode), n), S};
    ch = XArr<XChild>{(XChild*)take(sizeof(XChild), n), S};
    st_par = XArr<XStr>{(XStr*)take(sizeof(XStr), n), S};
    fr = XArr<XFrame>{(XFrame*)take(sizeof(XFrame), n), S};
    st_arr = XArr<uint8_t>{take(1, n), S};
    st_typ = XArr<uint8_t>{take(1, n), S};
    uint8_t* tabs = take(sizeof(uint32_t), 2ull * h);  // ht, then hc: 2h entries of one lane
    ht = XArr<uint32_t>{(uint32_t*)tabs, S};
    hc = XArr<uint32_t>{(uint32_t*)tabs + (uint64_t)h * S, S};
    nn_cap = nc_cap = st_cap = n;
    ht_mask = hc_mask = h - 1;
    if (S == 1) {
      // both tables cleared with 16-byte stores (adjacent, 16-aligned, h a multiple of 4): in the kernels every store
      // of a lane is a request of its own, and a dword-wise clear was a quarter of a small merge's requests
      struct alignas(16) Q { uint64_t a, b; };
      for (uint32_t i = 0; i < 2 * h; i += 4) *(Q*)((uint32_t*)tabs + i) = Q{0, 0};
    } else {
      for (uint32_t i = 0; i < 2 * h; i++) ht[i] = 0;  // (interleaved: the wave's lanes clear adjacent dwords)
    }
    // the lane's pool: its share of what the arrays leave (XPOOL_SLACK bytes kept free past it: the string helpers read
    // and write whole 8-byte chunks)
    const uint64_t pool_bytes = (((uint64_t)w.bytes * S - off) / S) & ~15ull;
    pool = w.base + off + (uint64_t)w.lane * pool_bytes;
    pool_cap = (uint32_t)pool_bytes - XPOOL_SLACK;
    pool_n = 0;
    nn = nc = 0;
    n_par = n_arr = n_typ = 0;
    typed[0] = typed[1] = 0;
    dollar = str_from((const uint8_t*)"$", 1);
    return status == X_OK;
  }

  // ---- strings, 8 bytes at a time (unaligned 8-byte accesses: a byte loop was one memory request per byte). A chunk
  // may read up to 7 bytes past a string (inside the pool's slack, or past a document: the arena keeps ARENA_SLACK
  // readable bytes) and a copy may write up to 7 bytes past it (free pool space above the top, overwritten later)
  ZB_HD static uint64_t ld8(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
  }
  ZB_HD static void st8(uint8_t* p, uint64_t v) { __builtin_memcpy(p, &v, 8); }
  ZB_HD static void copy8(uint8_t* d, const uint8_t* s, uint32_t n) {
    for (uint32_t i = 0; i < n; i += 8) st8(d + i, ld8(s + i));
  }
  ZB_HD XStr str_new(uint32_t len) {
    XStr r{pool_n, len};
    if ((uint64_t)pool_n + len > pool_cap) { status = X_UNSUP; r.len = 0; return r; }
    pool_n += len;
    return r;
  }
  ZB_HD XStr str_from(const uint8_t* p, uint32_t len) {
    XStr r = str_new(len);
    if (status == X_OK) copy8(pool + r.off, p, len);
    return r;
  }
  // MsgPackTreeNodeIdConstructor.construct: parent + "[" + name + "]" (at the pool's top: above both sources)
  ZB_HD XStr cat(XStr parent, XStr name) {
    XStr r = str_new(parent.len + name.len + 2);
    if (status != X_OK) return r;
    uint8_t* d = pool + r.off;
    copy8(d, pool + parent.off, parent.len);
    d[parent.len] = '[';
    copy8(d + parent.len + 1, pool + name.off, name.len);
    d[parent.len + 1 + name.len] = ']';
    return r;
  }
  ZB_HD XStr decimal(uint32_t v) {  // Integer.toString
    uint8_t t[10];
    uint32_t k = 0;
    do { t[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
    XStr r = str_new(k);
    if (status == X_OK)
      for (uint32_t i = 0; i < k; i++) pool[r.off + i] = t[k - 1 - i];
    return r;
  }
  ZB_HD bool eq(XStr a, XStr b) const {
    if (a.len != b.len) return false;
    for (uint32_t i = 0; i < a.len; i += 8) {
      uint64_t x = ld8(pool + a.off + i) ^ ld8(pool + b.off + i);
      if (a.len - i < 8) x &= ~0ull >> (64 - 8 * (a.len - i));
      if (x) return false;
    }
    return true;
  }
  ZB_HD uint32_t hash(XStr a, uint32_t seed) const {  // FNV-1a
    uint32_t h = 2166136261u ^ (seed * 0x9e3779b9u);
    for (uint32_t i = 0; i < a.len; i += 8) {
      uint64_t w = ld8(pool + a.off + i);
      const uint32_t m = a.len - i < 8 ? a.len - i : 8;
      for (uint32_t k = 0; k < m; k++, w >>= 8) h = (h ^ (uint32_t)(w & 0xff)) * 16777619u;
    }
    return h;
  }

  // ---- nodes by id
  ZB_HD uint32_t find(uint8_t tree, XStr id) const {
    const uint32_t h = hash(id, tree);
    for (uint32_t i = h & ht_mask;; i = (i + 1) & ht_mask) {
      const uint32_t e = ht[i];
      if (e == 0) return XNONE;
      const XNode& x = nodes[e - 1];
      if (x.hash == h && x.tree == tree && eq(x.id, id)) return e - 1;
    }
  }
  ZB_HD uint32_t get(uint8_t tree, XStr id) {
    const uint32_t h = hash(id, tree);
    uint32_t i = h & ht_mask;
    for (;; i = (i + 1) & ht_mask) {
      const uint32_t e = ht[i];
      if (e == 0) break;
      const XNode& x = nodes[e - 1];
      if (x.hash == h && x.tree == tree && eq(x.id, id)) return e - 1;
    }
    if (nn >= nn_cap) { status = X_UNSUP; return XNONE; }
    XNode& x = nodes[nn];
    x.id = id; x.hash = h; x.tree = tree; x.type = XT_NONE; x.has_leaf = 0; x.has_childs = 0;
    x.lpos = x.llen = 0; x.cfirst = x.clast = XNONE; x.ccount = 0;
    ht[i] = ++nn;
    return nn - 1;
  }
  ZB_HD void set_type(uint32_t x, uint8_t t) {
    if (nodes[x].type == XT_NONE) typed[nodes[x].tree]++;
    nodes[x].type = t;
  }

  // ---- MsgPackTree
  ZB_HD void add_leaf(uint8_t tree, XStr id, uint32_t pos, uint32_t len, bool extracting) {
    const uint32_t x = get(tree, id);
    if (x == XNONE) return;
    nodes[x].has_leaf = 1; nodes[x].lpos = pos; nodes[x].llen = len;
    set_type(x, extracting ? XT_EXTRACTED_LEAF : XT_EXISTING_LEAF);
  }
  ZB_HD void add_parent(uint8_t tree, XStr id, uint8_t t) {
    const uint32_t x = get(tree, id);
    if (x == XNONE) return;
    set_type(x, t);
    if (!nodes[x].has_childs) { nodes[x].has_childs = 1; nodes[x].cfirst = nodes[x].clast = XNONE; nodes[x].ccount = 0; }
  }
  ZB_HD void add_map(uint8_t tree, XStr id) {  // addMapNode: the leaf goes
    const uint32_t x = get(tree, id);
    if (x == XNONE) return;
    nodes[x].has_leaf = 0;
    add_parent(tree, id, XT_MAP);
  }
  ZB_HD void add_array(uint8_t tree, XStr id) { add_parent(tree, id, XT_ARRAY); }  // addArrayNode: the leaf stays
  ZB_HD bool is_map(uint8_t tree, XStr id) const {
    const uint32_t x = find(tree, id);
    return x != XNONE && nodes[x].type == XT_MAP;
  }
  // addChildToNode: nodeChildsMap.get(parent).add(name) -- a parent without a child set is a NullPointerException
  ZB_HD void add_child_to(uint32_t p, XStr name) {
    if (p == XNONE || !nodes[p].has_childs) { status = X_FAIL; return; }
    const uint32_t h = hash(name, p + 7);
    uint32_t i = h & hc_mask;
    for (;; i = (i + 1) & hc_mask) {
      const uint32_t e = hc[i];
      if (e == 0) break;
      const XChild& c = ch[e - 1];
      if (c.parent == p && eq(c.name, name)) return;  // LinkedHashSet.add of a member
    }
    if (nc >= nc_cap) { status = X_UNSUP; return; }
    XChild& c = ch[nc];
    c.name = name; c.next = XNONE; c.parent = p;
    hc[i] = ++nc;
    XNode& n = nodes[p];
    if (n.clast == XNONE) n.cfirst = nc - 1;
    else ch[n.clast].next = nc - 1;
    n.clast = nc - 1;
    n.ccount++;
  }
  ZB_HD void add_child(uint8_t tree, XStr name, XStr parent) { add_child_to(find(tree, parent), name); }

  // ---- MsgPackDocumentIndexer
  ZB_HD void push_par(XStr x) {
    if (n_par >= st_cap) { status = X_UNSUP; return; }
    st_par[n_par++] = x;
  }
  ZB_HD XStr pop_par() {
    if (n_par == 0) { status = X_FAIL; return XStr{0, 0}; }  // NoSuchElementException
    return st_par[--n_par];
  }
  ZB_HD void push_arr() {
    if (n_arr >= st_cap) { status = X_UNSUP; return; }
    st_arr[n_arr++] = 1;
  }
  ZB_HD void push_typ(uint8_t t) {
    if (n_typ >= st_cap) { status = X_UNSUP; return; }
    st_typ[n_typ++] = t;
  }

  ZB_HD void index(uint8_t tree, const uint8_t* d, uint32_t n, bool extracting) {
    n_par = n_arr = n_typ = 0;
    XStr last_key = dollar;
    uint8_t last_type = TT_EXTENSION;
    uint32_t pos = 0;
    while (pos < n && status == X_OK) {
      Tok t;
      if (!read_tok(d + pos, n - pos, t)) break;  // the reader's exception ends the traversal
      if (pos != 0 || t.type != TT_NIL) {
        last_type = n_typ ? st_typ[--n_typ] : (uint8_t)TT_EXTENSION;
        if (last_type == TT_MAP) {
          if (t.type != TT_STRING) { status = X_FAIL; return; }  // "non-string map key is not supported"
          last_key = str_from(d + pos + t.hdr, t.len);
          push_typ(TT_EXTENSION);
        } else if (t.type == TT_MAP || t.type == TT_ARRAY) {
          new_parent(tree, t.len, t.type, last_key, last_type);
        } else {
          value_node(tree, pos, t.total, last_key, last_type, extracting);
        }
      }
      pos += t.total;
    }
  }

  ZB_HD void new_parent(uint8_t tree, uint32_t count, uint8_t type, XStr name, uint8_t last_type) {
    XStr id;
    bool is_array_value;
    if (n_arr > 0) {
      is_array_value = st_arr[--n_arr] != 0;
      id = pop_par();
      if (last_type != TT_ARRAY) {
        push_par(id);
        id = cat(id, name);
      }
    } else {
      id = n_par == 0 ? name : cat(st_par[n_par - 1], name);
      is_array_value = false;
    }
    if (status != X_OK) return;
    if (type == TT_ARRAY) add_array(tree, id);
    else add_map(tree, id);
    if (n_par > 0 && last_type != TT_ARRAY) {
      const XStr parent = pop_par();
      add_child(tree, name, parent);
    }
    for (uint32_t i = 0; i < count && status == X_OK; i++) {
      if (type == TT_ARRAY) {
        add_child(tree, decimal(i), id);
        push_par(cat(id, decimal(count - 1 - i)));
        push_arr();
      } else {
        push_par(id);
        if (is_array_value) push_arr();
      }
      push_typ(type);
    }
  }

  ZB_HD void value_node(uint8_t tree, uint32_t pos, uint32_t len, XStr last_key, uint8_t last_type, bool extracting) {
    XStr parent = pop_par();
    if (status != X_OK) return;
    XStr name, id;
    if (n_arr > 0) {
      if (last_type != TT_ARRAY) {
        name = last_key;
        id = cat(parent, name);
      } else {
        // the element's own id: name = the text after the id's last '[', parent = the text before it
        id = parent;
        uint32_t li = XNONE;
        for (uint32_t k = parent.len; k > 0; k--)
          if (pool[parent.off + k - 1] == '[') { li = k - 1; break; }
        if (li != XNONE) {
          name = XStr{parent.off + li + 1, parent.len - li - 2};
          parent = XStr{parent.off, li};
        } else {
          name = XStr{parent.off, parent.len ? parent.len - 1 : 0};
        }
      }
      n_arr--;
    } else {
      name = last_key;
      id = cat(parent, name);
    }
    if (status != X_OK) return;
    add_child(tree, name, parent);
    add_leaf(tree, id, pos, len, extracting);
  }

  // ---- MsgPackTree.merge: the source tree's types (leaves become extracted), leaves and child sets; the root's
  // child set is the union, every other child set is replaced
  ZB_HD void merge_in() {
    const uint32_t n0 = nn;
    for (uint32_t i = 0; i < n0 && status == X_OK; i++) {
      if (nodes[i].tree != 1) continue;
      const XNode s = nodes[i];
      const uint32_t t = get(0, s.id);
      if (t == XNONE) return;
      if (s.type != XT_NONE) set_type(t, s.type == XT_EXISTING_LEAF ? XT_EXTRACTED_LEAF : s.type);
      if (s.has_leaf) { nodes[t].has_leaf = 1; nodes[t].lpos = s.lpos; nodes[t].llen = s.llen; }
      if (s.has_childs) {
        if (eq(s.id, dollar)) {
          if (!nodes[t].has_childs) { nodes[t].has_childs = 1; nodes[t].cfirst = nodes[t].clast = XNONE; nodes[t].ccount = 0; }
          for (uint32_t c = s.cfirst; c != XNONE && status == X_OK; c = ch[c].next) add_child_to(t, ch[c].name);
        } else {
          nodes[t].has_childs = 1;
          nodes[t].cfirst = s.cfirst; nodes[t].clast = s.clast; nodes[t].ccount = s.ccount;
        }
      }
    }
  }

  // ---- MsgPackDocumentTreeWriter over tree 0: leaves are read from the node type's buffer (extracted: x,
  // existing: u); o.n past limit stops it (X_UNSUP)
  template <class O>
  ZB_HD void node_out(XStr id, const uint8_t* u, uint32_t un, const uint8_t* x, uint32_t xn, O& o, uint32_t& depth) {
    const uint32_t k = find(0, id);
    if (k != XNONE && nodes[k].has_leaf) {
      const XNode& m = nodes[k];
      if (m.type == XT_NONE) { status = X_FAIL; return; }
      const bool ext = m.type == XT_EXTRACTED_LEAF;
      const uint8_t* b = ext ? x : u;
      const uint32_t bn = ext ? xn : un;
      if (!b || (uint64_t)m.lpos + m.llen > bn) { status = X_FAIL; return; }  // buffer bounds: IndexOutOfBounds
      o.put_bytes(b + m.lpos, m.llen);
      pool_n = id.off;  // (the id was the scratch top)
      return;
    }
    if (k == XNONE || !nodes[k].has_childs) { status = X_FAIL; return; }  // no child set: NullPointerException
    const bool arr = nodes[k].type == XT_ARRAY;
    if (arr) o.arr_hdr(nodes[k].ccount);
    else o.map_hdr(nodes[k].ccount);
    if (depth >= st_cap) { status = X_UNSUP; return; }
    fr[depth++] = XFrame{id, nodes[k].cfirst, arr ? 1u : 0u};
  }

  template <class O>
  ZB_HD void write(const uint8_t* u, uint32_t un, const uint8_t* x, uint32_t xn, O& o, uint32_t limit) {
    if (typed[0] == 0) { o.put(0xc0); return; }  // empty tree: writeNil
    const uint32_t mark = pool_n;
    uint32_t depth = 0;
    XStr root = str_from(dollar.off + pool, 1);
    if (status != X_OK) return;
    node_out(root, u, un, x, xn, o, depth);
    while (depth > 0 && status == X_OK) {
      if (o.n > limit) { status = X_UNSUP; break; }
      XFrame& f = fr[depth - 1];
      if (f.cur == XNONE) {
        pool_n = f.id.off;
        depth--;
        continue;
      }
      const XChild c = ch[f.cur];
      f.cur = c.next;
      if (!f.arr) o.str(s(c.name), c.name.len);
      const XStr id = cat(f.id, c.name);
      if (status != X_OK) break;
      node_out(id, u, un, x, xn, o, depth);
    }
    if (o.n > limit && status == X_OK) status = X_UNSUP;
    pool_n = mark;
  }

  // ensureDocumentIsAMsgPackMap on what write() produces: the root's leaf bytes or its container type
  ZB_HD int root_check(const uint8_t* u, const uint8_t* x) const {
    if (typed[0] == 0) return X_OK;  // nil
    const uint32_t k = find(0, dollar);
    if (k == XNONE) return X_FAIL;
    const XNode& m = nodes[k];
    if (m.has_leaf) {
      const uint8_t* d = m.type == XT_EXTRACTED_LEAF ? x : u;
      if (!d) return X_FAIL;
      const uint8_t b = d[m.lpos];
      return ((b & 0xf0) == 0x80 || b == 0xde || b == 0xdf || b == 0xc0) ? X_OK : X_NOT_MAP;
    }
    return m.type == XT_MAP ? X_OK : X_NOT_MAP;
  }
};

// tokens the indexer visits in a document (it stops at the first unreadable one)
ZB_HD inline uint32_t x_tokens(const uint8_t* d, uint32_t n) {
  uint32_t pos = 0, k = 0;
  while (pos < n) {
    Tok t;
    if (!read_tok(d + pos, n - pos, t)) break;
    pos += t.total;
    k++;
  }
  return k;
}

// A built tree written (o.dst set: one pass into o.dst that writes nothing at or past limit; an oversized result is
// X_UNSUP, as a size pass would have found it) or sized (o.dst null); the result must be a map or nil.
ZB_HD inline int x_emit(XTree& T, const uint8_t* u, uint32_t un, const uint8_t* x, uint32_t xn, Out& o, uint32_t limit) {
  if (o.dst) {
    OutCap oc{o.dst, 0, limit};
    T.write(u, un, x, xn, oc, limit);
    if (T.status != X_OK) return T.status;
    const int rc = T.root_check(u, x);
    if (rc != X_OK) return rc;
    o.n = oc.n;
    return X_OK;
  }
  Out sz{nullptr, 0};
  T.write(u, un, x, xn, sz, limit);
  if (T.status != X_OK) return T.status;
  const int rc = T.root_check(u, x);
  if (rc != X_OK) return rc;
  o.n = sz.n;
  return X_OK;
}

// MappingProcessor.merge(source, target) without mappings (has_tgt: the target buffer is not empty)
ZB_HD inline __noinline__ int x_merge(const XWs& ws, const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt,
                                      Out& o, uint32_t limit) {
  XTree T;
  // nodes / child entries / stack: each token makes at most one of each, the source's twice (merge_in)
  if (!T.init(ws, 2 * x_tokens(src, ns) + x_tokens(tgt, nt))) return T.status;
  if (nt == 0) {  // extract(source): index + write
    T.index(0, src, ns, false);
    if (T.status != X_OK) return T.status;
    return x_emit(T, src, ns, nullptr, 0, o, limit);
  }
  T.index(0, tgt, nt, false);
  if (T.status != X_OK) return T.status;
  T.index(1, src, ns, false);
  if (T.status != X_OK) return T.status;
  T.merge_in();
  if (T.status != X_OK) return T.status;
  return x_emit(T, tgt, nt, src, ns, o, limit);
}

// The tree of MappingProcessor.extract(source, mappings) (tgt == nullptr) or .merge(source, target, mappings) with
// nmaps >= 1, before it is written: the target indexed, then every mapping's target path and extracted leaf
ZB_HD inline int x_map_tree(XTree& T, const XWs& ws, const uint8_t* src, uint32_t ns,
                            const uint8_t* tgt, uint32_t nt, const DevMapping* maps, uint32_t nmaps, const DevSeg* segs,
                            const DevQuery* queries, const DevFilter* filters, const uint8_t* pool,
                            uint16_t& fail_query) {
  uint32_t segn = 0;
  for (uint32_t i = 0; i < nmaps; i++) segn += maps[i].nseg + 1;
  if (!T.init(ws, (tgt ? x_tokens(tgt, nt) : 0) + 2 * segn)) return T.status;
  if (tgt && nt) {
    T.index(0, tgt, nt, false);
    if (T.status != X_OK) return T.status;
  }
  for (uint32_t mi = 0; mi < nmaps; mi++) {
    const DevMapping m = maps[mi];
    XStr parent{0, 0};
    bool have = false;
    for (uint32_t k = 0; k < m.nseg; k++) {  // TargetPathVisitor: createParentRelation per literal
      const DevSeg sg = segs[m.seg + k];
      const XStr name = T.str_from(pool + sg.off, sg.len);
      if (T.status != X_OK) return T.status;
      if (!have) {
        parent = name;
        have = true;
        continue;
      }
      bool index = true;  // isIndex (an empty name counts as an index)
      for (uint32_t i = 0; i < sg.len; i++)
        if (pool[sg.off + i] < '0' || pool[sg.off + i] > '9') { index = false; break; }
      if (index) {
        if (!T.is_map(0, parent)) T.add_array(0, parent);
      } else {
        T.add_map(0, parent);
      }
      const XStr id = T.cat(parent, name);
      T.add_child(0, name, parent);
      if (T.status != X_OK) return T.status;
      parent = id;
    }
    QueryResult r;  // executeLeafMapping (the executor's per-depth state in the pool: any nesting depth)
    {
      const DevQuery& q = queries[m.query];
      if (q.fast) {
        if (!run_query(src, ns, q, filters, pool, r)) return X_UNSUP;
      } else {
        const uint32_t maxd = x_tokens(src, ns) + 1;
        const XStr w = T.str_new(maxd * 17 + 16);
        if (T.status != X_OK) return T.status;
        int* qi = (int*)(T.pool + ((w.off + 3) & ~3u));
        if (!query_walk(src, ns, filters + q.first, q.count, pool, r, qi, qi + maxd, qi + 2 * maxd, qi + 3 * maxd,
                        (bool*)(qi + 4 * maxd), (int)maxd))
          return X_UNSUP;
        T.pool_n = w.off;  // (scratch)
      }
    }
    if (r.count == 0) { fail_query = m.query; return X_NO_DATA; }
    if (r.count > 1) return X_FAIL;  // IllegalStateException: more than one matching source
    T.add_leaf(0, parent, r.pos, r.len, true);
    if (T.status != X_OK) return T.status;
  }
  return X_OK;
}

// MappingProcessor.extract(source, mappings) (tgt == nullptr) or .merge(source, target, mappings), nmaps >= 1
ZB_HD inline __noinline__ int x_map(const XWs& ws, const uint8_t* src, uint32_t ns, const uint8_t* tgt, uint32_t nt,
                                    const DevMapping* maps, uint32_t nmaps, const DevSeg* segs, const DevQuery* queries,
                                    const DevFilter* filters, const uint8_t* pool, Out& o, uint32_t limit,
                                    uint16_t& fail_query) {
  XTree T;
  const int st = x_map_tree(T, ws, src, ns, tgt, nt, maps, nmaps, segs, queries, filters, pool, fail_query);
  if (st != X_OK) return st;
  return x_emit(T, tgt, tgt ? nt : 0, src, ns, o, limit);
}

}  // namespace zbg
