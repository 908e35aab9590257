// ORACLE / TEST INFRASTRUCTURE ONLY. Never linked into the product (zeebe_amd/csrc).
//
// Default (mapping-less) payload merge, restated literally from the reference, including its
// string node ids and LinkedHashSet child order:
//   MappingProcessor.merge:        json-path/src/main/java/io/zeebe/msgpack/mapping/MappingProcessor.java:143-170,206-223
//   MsgPackDocumentIndexer:        json-path/src/main/java/io/zeebe/msgpack/mapping/MsgPackDocumentIndexer.java:136-283
//   MsgPackTree (+ merge):         json-path/src/main/java/io/zeebe/msgpack/mapping/MsgPackTree.java:84-166
//   MsgPackDocumentTreeWriter:     json-path/src/main/java/io/zeebe/msgpack/mapping/MsgPackDocumentTreeWriter.java:53-104
//   node ids:                      json-path/src/main/java/io/zeebe/msgpack/mapping/MsgPackTreeNodeIdConstructor.java
#pragma once
#include <deque>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "zbref_jsonpath.hpp"
#include "zbref_msgpack.hpp"

namespace zbref {

struct MappingError : std::runtime_error {  // MappingException
  using std::runtime_error::runtime_error;
};

inline std::string node_id(const std::string& parent, const std::string& name) { return parent + "[" + name + "]"; }

struct LinkedSet {  // java.util.LinkedHashSet<String>
  std::vector<std::string> order;
  std::unordered_set<std::string> members;
  void add(const std::string& s) {
    if (members.insert(s).second) order.push_back(s);
  }
};

enum class NodeType { EXISTING_LEAF, EXTRACTED_LEAF, MAP, ARRAY };

struct MsgPackTree {
  std::unordered_map<std::string, NodeType> node_type;
  std::unordered_map<std::string, LinkedSet> childs;
  std::unordered_map<std::string, uint64_t> leaf;
  bytes underlying;
  const bytes* extract = nullptr;

  void add_leaf(const std::string& id, uint32_t pos, uint32_t len) {
    leaf[id] = ((uint64_t)pos << 32) | len;
    node_type[id] = extract == nullptr ? NodeType::EXISTING_LEAF : NodeType::EXTRACTED_LEAF;
  }
  void add_parent(const std::string& id, NodeType t) {
    node_type[id] = t;
    if (!childs.count(id)) childs[id] = LinkedSet();
  }
  void add_map(const std::string& id) {
    if (leaf.count(id)) leaf.erase(id);
    add_parent(id, NodeType::MAP);
  }
  void add_array(const std::string& id) { add_parent(id, NodeType::ARRAY); }
  void add_child(const std::string& name, const std::string& parent) { childs.at(parent).add(name); }
  bool is_leaf(const std::string& id) const { return leaf.count(id) != 0; }
  bool is_array(const std::string& id) const {
    auto it = node_type.find(id);
    return it != node_type.end() && it->second == NodeType::ARRAY;
  }
  bool is_map(const std::string& id) const {
    auto it = node_type.find(id);
    return it != node_type.end() && it->second == NodeType::MAP;
  }

  // MsgPackTree.merge :141-166 (top-level merge: only the root child set is unioned)
  void merge(const MsgPackTree& src) {
    extract = &src.underlying;
    for (auto& kv : src.node_type) {
      NodeType t = kv.second == NodeType::EXISTING_LEAF ? NodeType::EXTRACTED_LEAF : kv.second;
      node_type[kv.first] = t;
    }
    for (auto& kv : src.leaf) leaf[kv.first] = kv.second;
    for (auto& kv : src.childs) {
      if (kv.first == "$") {
        LinkedSet& dst = childs["$"];
        for (auto& c : kv.second.order) dst.add(c);
      } else {
        childs[kv.first] = kv.second;
      }
    }
  }
};

// MsgPackDocumentIndexer: a literal restatement of its stack machine
struct DocumentIndexer {
  MsgPackTree* tree;
  std::string last_key = "$";
  MpType last_type = MpType::EXTENSION;
  std::deque<std::string> parents;     // ArrayDeque used as a stack (push/pop/peek at front)
  std::deque<bool> array_values;
  std::deque<MpType> last_types;

  MpType pop_last_type() {
    if (last_types.empty()) return MpType::EXTENSION;
    MpType t = last_types.front();
    last_types.pop_front();
    return t;
  }
  std::string pop_parent() {
    if (parents.empty()) throw ZbError("NoSuchElementException");
    std::string p = parents.front();
    parents.pop_front();
    return p;
  }

  void visit(uint32_t position, const MpToken& tok) {
    if (position != 0 || tok.type != MpType::NIL) {
      last_type = pop_last_type();
      if (last_type == MpType::MAP) {
        if (tok.type != MpType::STRING) throw ZbError("non-string map key is not supported");
        last_key = tok.value();
        last_types.push_front(MpType::EXTENSION);
      } else if (tok.type == MpType::MAP || tok.type == MpType::ARRAY) {
        add_new_parent(tok.size, tok.type);
      } else {
        process_value(position, tok);
      }
    }
  }

  void add_new_parent(uint32_t child_count, MpType type) {
    std::string name = last_key;
    std::string id;
    bool is_array_value;
    if (!array_values.empty()) {
      is_array_value = array_values.front();
      array_values.pop_front();
      id = pop_parent();
      if (last_type != MpType::ARRAY) {
        parents.push_front(id);
        id = node_id(id, name);
      }
    } else {
      id = parents.empty() ? name : node_id(parents.front(), name);
      is_array_value = false;
    }
    // addParentNodeToTree
    if (type == MpType::ARRAY) tree->add_array(id);
    else tree->add_map(id);
    if (!parents.empty() && last_type != MpType::ARRAY) {
      std::string parent = pop_parent();
      tree->add_child(name, parent);
    }
    // addParentForChildCountToStacks
    for (uint32_t i = 0; i < child_count; i++) {
      if (type == MpType::ARRAY) {
        tree->add_child(std::to_string(i), id);
        parents.push_front(node_id(id, std::to_string(child_count - 1 - i)));
        array_values.push_front(true);
      } else {
        parents.push_front(id);
        if (is_array_value) array_values.push_front(true);
      }
      last_types.push_front(type);
    }
  }

  void process_value(uint32_t position, const MpToken& tok) {
    std::string parent = pop_parent();
    std::string name, id;
    if (!array_values.empty()) {
      if (last_type != MpType::ARRAY) {
        name = last_key;
        id = node_id(parent, name);
      } else {
        id = parent;
        size_t li = parent.rfind('[');
        name = parent.substr(li + 1, parent.size() - 1 - (li + 1));
        parent = parent.substr(0, li);
      }
      array_values.pop_front();
    } else {
      name = last_key;
      id = node_id(parent, name);
    }
    tree->add_child(name, parent);
    tree->add_leaf(id, position, tok.total);
  }

  void index(MsgPackTree& t, const bytes& doc) {
    tree = &t;
    t.node_type.clear(); t.childs.clear(); t.leaf.clear(); t.extract = nullptr;
    t.underlying = doc;
    MpReader r(doc);
    while (r.has_next()) {
      uint32_t pos = (uint32_t)r.off;
      MpToken tok;
      try {
        tok = r.read_token();
      } catch (const ZbError&) {
        break;
      }
      visit(pos, tok);
    }
  }
};

struct TreeWriter {
  const MsgPackTree* t;
  MpWriter w;
  void write_node(const std::string& parent, const std::string& name, bool is_array) {
    if (!parent.empty() && !is_array) w.str(name);
    std::string id = parent.empty() ? name : node_id(parent, name);
    if (t->is_leaf(id)) {
      uint64_t m = t->leaf.at(id);
      uint32_t pos = (uint32_t)(m >> 32), len = (uint32_t)m;
      NodeType nt = t->node_type.at(id);
      const bytes& buf = (nt == NodeType::EXTRACTED_LEAF) ? *t->extract : t->underlying;
      // the buffer follows the node type (an extracted leaf whose node addArrayNode retyped is read from the
      // indexed document); UnsafeBuffer bounds checks throw outside it
      if ((size_t)pos + len > buf.size()) throw ZbError("IndexOutOfBoundsException in tree writer");
      w.raw(buf.data() + pos, len);
    } else {
      bool arr = t->is_array(id);
      auto it = t->childs.find(id);
      if (it == t->childs.end()) throw ZbError("NullPointerException in tree writer");
      const LinkedSet& cs = it->second;
      if (arr) w.array_header((uint32_t)cs.order.size());
      else w.map_header((uint32_t)cs.order.size());
      for (auto& c : cs.order) write_node(id, c, arr);
    }
  }
  bytes write(const MsgPackTree& tree) {
    t = &tree;
    w.b.clear();
    if (!tree.node_type.empty()) write_node("", "$", false);
    else w.nil();
    return w.b;
  }
};

// MappingProcessor.merge(source, target) with no mappings
inline bytes merge_documents(const bytes& source, const bytes& target) {
  if (target.empty()) {
    // extract(source) without mappings = index + rewrite
    MsgPackTree t;
    DocumentIndexer ix;
    ix.index(t, source);
    TreeWriter tw;
    bytes out = tw.write(t);
    MpType ty = mp_format_type((uint8_t)out[0]);
    if (ty != MpType::MAP && ty != MpType::NIL)
      throw MappingError("Processing failed, since mapping will result in a non map object (json object).");
    return out;
  }
  MsgPackTree tgt, src;
  DocumentIndexer ix1, ix2;
  ix1.index(tgt, target);
  ix2.index(src, source);
  tgt.merge(src);
  TreeWriter tw;
  bytes out = tw.write(tgt);
  MpType ty = mp_format_type((uint8_t)out[0]);
  if (ty != MpType::MAP && ty != MpType::NIL)
    throw MappingError("Processing failed, since mapping will result in a non map object (json object).");
  return out;
}

// ------------------------------------------------------------------------------ explicit mappings
// Mapping (json-path/.../mapping/Mapping.java): a compiled source query and a target path.
struct Mapping {
  JsonPathQuery source;
  bytes target;
};

inline void ensure_map_result(const bytes& out) {  // MappingProcessor.ensureDocumentIsAMsgPackMap :206-213
  MpType ty = mp_format_type((uint8_t)out[0]);
  if (ty != MpType::MAP && ty != MpType::NIL)
    throw MappingError("Processing failed, since mapping will result in a non map object (json object).");
}

// MsgPackDocumentExtractor.createParentRelation :146-166
inline std::string create_parent_relation(MsgPackTree& t, const std::string& parent, const std::string& name) {
  if (parent.empty()) return name;
  bool is_index = true;  // isIndex :168-177 (an empty name counts as an index)
  for (char c : name)
    if (c < '0' || c > '9') { is_index = false; break; }
  if (is_index) {
    if (!t.is_map(parent)) t.add_array(parent);
  } else {
    t.add_map(parent);
  }
  std::string id = node_id(parent, name);
  t.add_child(name, parent);
  return id;
}

// MsgPackDocumentExtractor.extract :121-128 with TargetPathVisitor :205-228 and executeLeafMapping :185-203
inline void extract_mappings(MsgPackTree& t, const bytes& doc, const std::vector<Mapping>& mappings) {
  t.extract = &doc;  // setExtractDocument
  for (const Mapping& m : mappings) {
    std::string node, parent;
    jp_tokenize(m.target, [&](JpToken type, int off, int len) {
      if (type == JpToken::LITERAL || type == JpToken::ROOT_OBJECT) {
        node = create_parent_relation(t, parent, m.target.substr(off, len));
        parent = node;
      } else if (type == JpToken::END_INPUT) {
        JsonPathExecutor ex;
        ex.run(m.source.filters, (const uint8_t*)doc.data(), doc.size());
        if (ex.results.empty())
          throw MappingError("No data found for query " + m.source.expression + ".");
        if (ex.results.size() > 1)  // IllegalStateException: not a MappingException, the processor fails
          throw ZbError("JSON path mapping has more than one matching source.");
        t.add_leaf(node, (uint32_t)ex.results[0].position, (uint32_t)ex.results[0].length);
      }
    });
  }
}

// MappingProcessor.extract :179-190
inline bytes map_extract(const bytes& source, const std::vector<Mapping>& mappings) {
  MsgPackTree t;
  if (mappings.empty()) {
    DocumentIndexer ix;
    ix.index(t, source);
  } else {
    extract_mappings(t, source, mappings);
  }
  TreeWriter tw;
  bytes out = tw.write(t);
  ensure_map_result(out);
  return out;
}

// MappingProcessor.merge :143-170 (the target is indexed, then the mappings extract into its tree)
inline bytes map_merge(const bytes& source, const bytes& target, const std::vector<Mapping>& mappings) {
  if (mappings.empty()) return merge_documents(source, target);
  if (target.empty()) return map_extract(source, mappings);
  MsgPackTree t;
  DocumentIndexer ix;
  ix.index(t, target);
  extract_mappings(t, source, mappings);
  TreeWriter tw;
  bytes out = tw.write(t);
  ensure_map_result(out);
  return out;
}

}  // namespace zbref
