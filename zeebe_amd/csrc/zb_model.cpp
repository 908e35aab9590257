// zb_model.cpp — BPMN XML -> device tables (see zb_model.hpp for the reference semantics followed).
#include "zb_model.hpp"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <unordered_map>

namespace zbg {

uint32_t ModelTables::add_bytes(const std::string& s) {
  uint32_t off = (uint32_t)pool.size();
  pool.insert(pool.end(), s.begin(), s.end());
  return off;
}

namespace {

// ------------------------------------------------------------------ a small DOM
struct Node {
  std::string tag;  // local name
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<Node>> kids;
  std::string text;
  Node* up = nullptr;
  const char* get(const char* k) const {
    for (auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
};

struct XmlError {
  std::string msg;
};

std::string strip_prefix(const std::string& n) {
  size_t c = n.rfind(':');
  return c == std::string::npos ? n : n.substr(c + 1);
}

void append_utf8(std::string& o, uint32_t c) {
  if (c < 0x80) { o += (char)c; return; }
  if (c < 0x800) { o += (char)(0xc0 | (c >> 6)); o += (char)(0x80 | (c & 63)); return; }
  if (c < 0x10000) {
    o += (char)(0xe0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63));
    return;
  }
  o += (char)(0xf0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 63));
  o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63));
}

std::string unescape(const char* b, const char* e) {
  std::string o;
  o.reserve(e - b);
  while (b < e) {
    if (*b != '&') { o += *b++; continue; }
    const char* semi = (const char*)memchr(b, ';', e - b);
    if (!semi) { o += *b++; continue; }
    std::string ent(b + 1, semi);
    if (ent == "amp") o += '&';
    else if (ent == "lt") o += '<';
    else if (ent == "gt") o += '>';
    else if (ent == "quot") o += '"';
    else if (ent == "apos") o += '\'';
    else if (ent.size() > 1 && ent[0] == '#')
      append_utf8(o, (uint32_t)strtoul(ent.c_str() + (ent[1] == 'x' || ent[1] == 'X' ? 2 : 1), nullptr,
                                       ent[1] == 'x' || ent[1] == 'X' ? 16 : 10));
    else o.append(b, semi + 1);
    b = semi + 1;
  }
  return o;
}

std::unique_ptr<Node> parse_xml(const std::string& doc) {
  auto root = std::make_unique<Node>();
  root->tag = "#root";
  Node* cur = root.get();
  const char* p = doc.data();
  const char* end = p + doc.size();
  auto fail = [](const char* m) { throw XmlError{m}; };
  while (p < end) {
    if (*p != '<') {
      const char* q = (const char*)memchr(p, '<', end - p);
      if (!q) q = end;
      cur->text += unescape(p, q);
      p = q;
      continue;
    }
    if (end - p >= 4 && !memcmp(p, "<!--", 4)) {
      const char* q = strstr(p + 4, "-->");
      if (!q) fail("unterminated comment");
      p = q + 3;
    } else if (end - p >= 9 && !memcmp(p, "<![CDATA[", 9)) {
      const char* q = strstr(p + 9, "]]>");
      if (!q) fail("unterminated CDATA");
      cur->text.append(p + 9, q);
      p = q + 3;
    } else if (end - p >= 2 && (p[1] == '?' || p[1] == '!')) {
      const char* q = (const char*)memchr(p, '>', end - p);
      if (!q) fail("unterminated declaration");
      p = q + 1;
    } else if (end - p >= 2 && p[1] == '/') {
      const char* q = (const char*)memchr(p, '>', end - p);
      if (!q || !cur->up) fail("bad end tag");
      cur = cur->up;
      p = q + 1;
    } else {
      ++p;
      const char* n0 = p;
      while (p < end && !strchr(" \t\r\n/>", *p)) ++p;
      auto node = std::make_unique<Node>();
      node->tag = strip_prefix(std::string(n0, p));
      node->up = cur;
      bool closed = false;
      for (;;) {
        while (p < end && strchr(" \t\r\n", *p)) ++p;
        if (p >= end) fail("unterminated tag");
        if (*p == '>') { ++p; break; }
        if (*p == '/') { closed = true; ++p; continue; }
        const char* a0 = p;
        while (p < end && !strchr(" \t\r\n=/>", *p)) ++p;
        std::string an(a0, p);
        while (p < end && strchr(" \t\r\n", *p)) ++p;
        if (p >= end || *p != '=') fail("attribute without value");
        ++p;
        while (p < end && strchr(" \t\r\n", *p)) ++p;
        if (p >= end || (*p != '"' && *p != '\'')) fail("unquoted attribute");
        char qc = *p++;
        const char* v0 = p;
        const char* v1 = (const char*)memchr(p, qc, end - p);
        if (!v1) fail("unterminated attribute value");
        p = v1 + 1;
        if (an == "xmlns" || an.compare(0, 6, "xmlns:") == 0) continue;
        node->attrs.emplace_back(strip_prefix(an), unescape(v0, v1));
      }
      Node* raw = node.get();
      cur->kids.push_back(std::move(node));
      if (!closed) cur = raw;
    }
  }
  if (cur != root.get()) fail("unclosed element");
  return root;
}

// ------------------------------------------------------------------ json-path compiler
bool compile_filters(const std::string& e, std::vector<DevFilter>& out, ModelTables& t, std::string& err) {
  // JsonPathTokenizer.java:59-106 static tokens, tried in this order at every position
  static const char* TOK[8] = {"$", "..", ".", "*", "['", "']", "[", "]"};
  enum { T_ROOT, T_REC, T_CHILD, T_WILD, T_CB_BEGIN, T_CB_END, T_SUB_BEGIN, T_SUB_END, T_LIT };
  bool subordinate = false;
  bool invalid = false;
  auto visit = [&](int tok, size_t off, size_t len) {
    if (invalid) return;
    if (!subordinate) {
      if (tok == T_ROOT) { DevFilter f{}; f.id = F_ROOT; out.push_back(f); }
      else if (tok == T_CHILD || tok == T_SUB_BEGIN || tok == T_CB_BEGIN) subordinate = true;
      else if (tok == T_SUB_END || tok == T_CB_END) {}
      else {
        invalid = true;
        static const char* NAMES[9] = {"ROOT_OBJECT", "RECURSION_OPERATOR", "CHILD_OPERATOR", "WILDCARD",
                                       "CHILD_BRACKET_OPERATOR_BEGIN", "CHILD_BRACKET_OPERATOR_END",
                                       "SUBSCRIPT_OPERATOR_BEGIN", "SUBSCRIPT_OPERATOR_END", "LITERAL"};
        err = std::string("Unexpected json-path token ") + NAMES[tok];
      }
      return;
    }
    if (tok == T_LIT) {
      bool digits = true;
      for (size_t i = off; i < off + len; i++)
        if ((signed char)e[i] < '0' || (signed char)e[i] > '9') digits = false;
      DevFilter f{};
      if (digits) {
        uint32_t v = 0, m = 1;  // ByteUtil.parseInteger (32-bit wraparound)
        for (size_t i = len; i-- > 0;) { v += (uint32_t)(e[off + i] - '0') * m; m *= 10u; }
        f.id = F_INDEX;
        f.index = (int32_t)v;
      } else {
        f.id = F_MAP_KEY;
        f.key_off = t.add_bytes(e.substr(off, len));
        f.key_len = (uint16_t)len;
      }
      out.push_back(f);
      subordinate = false;
    } else if (tok == T_WILD) {
      DevFilter f{};
      f.id = F_WILDCARD;
      out.push_back(f);
    } else {
      invalid = true;
      static const char* NAMES[9] = {"ROOT_OBJECT", "RECURSION_OPERATOR", "CHILD_OPERATOR", "WILDCARD",
                                     "CHILD_BRACKET_OPERATOR_BEGIN", "CHILD_BRACKET_OPERATOR_END",
                                     "SUBSCRIPT_OPERATOR_BEGIN", "SUBSCRIPT_OPERATOR_END", "LITERAL"};
      err = std::string("Unexpected json-path token ") + NAMES[tok];
    }
  };
  size_t pos = 0, lit0 = 0;
  bool bracket = false;
  while (pos < e.size()) {
    int hit = -1;
    for (int i = 0; i < 8 && hit < 0; i++) {
      if (bracket && i != T_CB_END) continue;
      size_t n = strlen(TOK[i]);
      if (e.compare(pos, n, TOK[i]) == 0) hit = i;
    }
    if (hit < 0) { pos++; continue; }
    if (lit0 < pos) visit(T_LIT, lit0, pos - lit0);
    bracket = hit == T_CB_BEGIN;
    visit(hit, pos, strlen(TOK[hit]));
    pos += strlen(TOK[hit]);
    lit0 = pos;
  }
  if (lit0 < pos) visit(T_LIT, lit0, pos - lit0);
  return !invalid;
}

// ------------------------------------------------------------------ json-el compiler
struct CondAst {
  int op;  // 0..5 comparison (CmpOp), 10 AND, 11 OR
  int lhs_path = 0, rhs_path = 0, lhs = 0, rhs = 0;
  std::unique_ptr<CondAst> l, r;
};

class CondParser {
 public:
  CondParser(const std::string& s, ModelTables& t) : s_(s), t_(t) {}
  // JsonConditionParser.parse = parseAll(condition): a committed failure (after `~!`) is final; otherwise
  // the message is the furthest failure recorded while parsing, the later one at equal positions
  // (scala-parser-combinators 1.0.6 lastNoSuccessVar; RegexParsers.phrase appends opt("\z"))
  std::unique_ptr<CondAst> parse(std::string& err) {
    size_t p = 0;
    auto c = condition(p);
    if (committed_) { err = err_; return nullptr; }
    if (!c) { err = rec_msg_; return nullptr; }
    const size_t q = ws(p);
    if (q != s_.size()) {
      record("string matching regex `\\z' expected but " + found(q) + " found", q);
      err = (rec_set_ && rec_pos_ >= p) ? rec_msg_ : "end of input expected";
      return nullptr;
    }
    return c;
  }

 private:
  const std::string& s_;
  ModelTables& t_;
  std::string err_;
  bool committed_ = false;
  std::string rec_msg_;
  size_t rec_pos_ = 0;
  bool rec_set_ = false;

  void record(const std::string& m, size_t pos) {  // NoSuccess: furthest wins, the later at a tie
    if (!rec_set_ || pos >= rec_pos_) { rec_msg_ = m; rec_pos_ = pos; rec_set_ = true; }
  }
  std::string found(size_t p) const {
    if (p >= s_.size()) return "end of source";
    return std::string("`") + s_[p] + "'";
  }
  // condition = disjunction | failure("expected comparison, disjunction or conjunction.")
  std::unique_ptr<CondAst> condition(size_t& p) {
    const size_t p0 = p;
    auto c = disjunction(p);
    if (!c && !committed_) record("expected comparison, disjunction or conjunction.", p0);
    return c;
  }

  size_t ws(size_t p) const {
    while (p < s_.size() && strchr(" \t\r\n\f\v", s_[p]) && s_[p]) p++;
    return p;
  }
  bool lit(size_t& p, const char* l) {
    size_t q = ws(p), n = strlen(l);
    if (s_.compare(q, n, l) == 0) { p = q + n; return true; }
    return false;
  }
  // operand: returns kind (0 const, 1 path), index; allow_all=false restricts to number|path
  bool operand(size_t& p, bool allow_all, int& is_path, int& idx) {
    size_t q = ws(p);
    if (q < s_.size() && s_[q] == '$') {  // \$([^\s])*
      size_t e = q + 1;
      while (e < s_.size() && !strchr(" \t\r\n\f\v", s_[e])) e++;
      std::string perr;
      int qi = compile_query(t_, s_.substr(q, e - q), perr);
      if (qi < 0) { err_ = perr; committed_ = true; return false; }
      is_path = 1; idx = qi; p = e;
      return true;
    }
    DevConst c{};
    if (allow_all && q < s_.size() && (s_[q] == '"' || s_[q] == '\'')) {
      // JsonConditionParser.string: JavaTokenParsers.stringLiteral "([^"\x00-\x1F\x7F\\]|\\[\\'"bfnrt]|
      // \\u[a-fA-F0-9]{4})*" or the same between single quotes without '"'; the body is kept raw
      const char qc = s_[q];
      size_t e = q + 1;
      while (e < s_.size() && s_[e] != qc) {
        const unsigned char ch = (unsigned char)s_[e];
        if (ch < 0x20 || ch == 0x7f || (qc == '\'' && ch == '"')) break;
        if (ch == '\\') {
          if (e + 1 < s_.size() && strchr("\\'\"bfnrt", s_[e + 1]) && s_[e + 1] != 0) { e += 2; continue; }
          if (e + 5 < s_.size() && s_[e + 1] == 'u' && isxdigit((unsigned char)s_[e + 2]) &&
              isxdigit((unsigned char)s_[e + 3]) && isxdigit((unsigned char)s_[e + 4]) &&
              isxdigit((unsigned char)s_[e + 5])) { e += 6; continue; }
          break;
        }
        e++;
      }
      if (e >= s_.size() || s_[e] != qc) return false;
      std::string body = s_.substr(q + 1, e - q - 1);  // kept raw (no unescaping), as the reference
      c.type = TT_STRING;
      c.str_off = t_.add_bytes(body);
      c.str_len = (uint16_t)body.size();
      p = e + 1;
    } else if (number(q, c, p)) {
    } else if (allow_all && s_.compare(q, 4, "true") == 0) { c.type = TT_BOOLEAN; c.bval = 1; p = q + 4; }
    else if (allow_all && s_.compare(q, 5, "false") == 0) { c.type = TT_BOOLEAN; c.bval = 0; p = q + 5; }
    else if (allow_all && s_.compare(q, 4, "null") == 0) { c.type = TT_NIL; p = q + 4; }
    else return false;
    is_path = 0;
    idx = (int)t_.consts.size();
    t_.consts.push_back(c);
    return true;
  }
  bool number(size_t q, DevConst& c, size_t& p) {
    size_t i = q;
    if (i < s_.size() && s_[i] == '-') i++;
    size_t d0 = i;
    while (i < s_.size() && isdigit((unsigned char)s_[i])) i++;
    size_t nint = i - d0;
    if (i < s_.size() && s_[i] == '.') {
      size_t j = i + 1;
      while (j < s_.size() && isdigit((unsigned char)s_[j])) j++;
      if (nint + (j - i - 1) > 0) {
        size_t e = j;
        if (e < s_.size() && (s_[e] == 'e' || s_[e] == 'E')) {
          size_t k = e + 1;
          if (k < s_.size() && (s_[k] == '+' || s_[k] == '-')) k++;
          size_t k0 = k;
          while (k < s_.size() && isdigit((unsigned char)s_[k])) k++;
          if (k > k0) e = k;
        }
        std::string num = s_.substr(q, e - q);
        if (e < s_.size() && strchr("fFdD", s_[e]) && s_[e]) e++;
        c.type = TT_FLOAT;
        c.fval = strtod(num.c_str(), nullptr);
        p = e;
        return true;
      }
    }
    if (nint == 0) return false;
    c.type = TT_INTEGER;
    c.ival = strtoll(s_.substr(q, i - q).c_str(), nullptr, 10);
    p = i;
    return true;
  }
  std::unique_ptr<CondAst> comparison(size_t& p) {
    size_t save = p;
    size_t reach = ws(p);  // furthest position its alternatives got to (withFailureMessage keeps it)
    int lp, li;
    if (operand(p, true, lp, li)) {
      size_t q = p;
      reach = ws(p);
      int op = -1;
      if (lit(q, "==")) op = OP_EQ;
      else if (lit(q, "!=")) op = OP_NE;
      if (op >= 0) {
        int rp, ri;
        if (!operand(q, true, rp, ri)) {
          committed_ = true;
          if (err_.empty()) err_ = "expected literal (JSON path, string, number, boolean, null)";
          return nullptr;
        }
        auto n = std::make_unique<CondAst>();
        n->op = op; n->lhs_path = lp; n->lhs = li; n->rhs_path = rp; n->rhs = ri;
        p = q;
        return n;
      }
      // number | path for ordering comparisons
      const DevConst* lc = lp ? nullptr : &t_.consts[li];
      if (lp || lc->type == TT_INTEGER || lc->type == TT_FLOAT) {
        static const char* OPS[4] = {"<=", ">=", "<", ">"};
        static const int OPV[4] = {OP_LE, OP_GE, OP_LT, OP_GT};
        for (int k = 0; k < 4; k++) {
          size_t r = p;
          if (lit(r, OPS[k])) {
            int rp, ri;
            if (!operand(r, false, rp, ri)) {
              committed_ = true;
              if (err_.empty()) err_ = "expected number or JSON path";
              return nullptr;
            }
            auto n = std::make_unique<CondAst>();
            n->op = OPV[k]; n->lhs_path = lp; n->lhs = li; n->rhs_path = rp; n->rhs = ri;
            p = r;
            return n;
          }
        }
      }
      if (committed_) return nullptr;
      p = save;
    }
    if (committed_) return nullptr;
    size_t q = p;
    if (lit(q, "(")) {  // "(" ~! condition ~ ")": everything after "(" is committed
      auto c = condition(q);
      if (!c) { committed_ = true; if (err_.empty()) err_ = rec_msg_; return nullptr; }
      if (!lit(q, ")")) {
        committed_ = true;
        if (err_.empty()) err_ = "`)' expected but " + found(ws(q)) + " found";
        return nullptr;
      }
      p = q;
      return c;
    }
    record("expected comparison operator ('==', '!=', '<', '<=', '>', '>=')", reach);
    return nullptr;
  }
  // chainl1(comparison | failure("expected comparison"), "&&")
  std::unique_ptr<CondAst> comparison_or_fail(size_t& p) {
    const size_t p0 = p;
    auto c = comparison(p);
    if (!c && !committed_) record("expected comparison", p0);
    return c;
  }
  std::unique_ptr<CondAst> conjunction(size_t& p) {
    auto l = comparison_or_fail(p);
    if (!l) return nullptr;
    for (;;) {
      size_t q = p;
      if (!lit(q, "&&")) break;
      auto r = comparison_or_fail(q);
      if (!r) {
        if (committed_) return nullptr;
        break;
      }
      auto n = std::make_unique<CondAst>();
      n->op = 10; n->l = std::move(l); n->r = std::move(r);
      l = std::move(n);
      p = q;
    }
    return l;
  }
  std::unique_ptr<CondAst> disjunction(size_t& p) {
    auto l = conjunction(p);
    if (!l) return nullptr;
    for (;;) {
      size_t q = p;
      if (!lit(q, "||")) break;
      auto r = conjunction(q);
      if (!r) {
        if (committed_) return nullptr;
        break;
      }
      auto n = std::make_unique<CondAst>();
      n->op = 11; n->l = std::move(l); n->r = std::move(r);
      l = std::move(n);
      p = q;
    }
    return l;
  }
};

void emit(ModelTables& t, const CondAst* n) {
  if (n->op == 10 || n->op == 11) {
    emit(t, n->l.get());
    size_t jump = t.code.size();
    t.code.push_back(n->op == 10 ? PC_JF : PC_JT);
    t.code.push_back(0);
    emit(t, n->r.get());
    uint32_t target = (uint32_t)(t.code.size() / 2);  // absolute instruction index
    t.code[jump] |= target << 16;
    return;
  }
  t.code.push_back((uint32_t)PC_CMP | ((uint32_t)n->op << 8) | ((uint32_t)n->lhs_path << 12) |
                   ((uint32_t)n->rhs_path << 13));
  t.code.push_back((uint32_t)n->lhs | ((uint32_t)n->rhs << 16));
}

// ------------------------------------------------------------------ transformer
bool is_flow_node_tag(const std::string& n) {
  static const char* T[] = {"startEvent", "endEvent", "serviceTask", "subProcess", "exclusiveGateway",
                            "intermediateCatchEvent", "parallelGateway", "inclusiveGateway", "eventBasedGateway",
                            "complexGateway", "task", "userTask", "receiveTask", "sendTask", "scriptTask",
                            "businessRuleTask", "manualTask", "callActivity", "transaction",
                            "intermediateThrowEvent", "boundaryEvent"};
  for (auto* x : T)
    if (n == x) return true;
  return false;
}

const Node* child(const Node* n, const char* tag) {
  for (auto& k : n->kids)
    if (k->tag == tag) return k.get();
  return nullptr;
}
const Node* extension(const Node* n, const char* tag) {
  for (auto& k : n->kids)
    if (k->tag == "extensionElements")
      if (const Node* c = child(k.get(), tag)) return c;
  return nullptr;
}
std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && strchr(" \t\r\n", s[b])) b++;
  while (e > b && strchr(" \t\r\n", s[e - 1])) e--;
  return s.substr(b, e - b);
}

struct Deployer {
  ModelTables& t;
  std::string& err;
  std::unordered_map<std::string, const Node*> dom_ids;
  // per process being compiled
  std::unordered_map<std::string, uint16_t> ids;  // element id -> global index
  uint16_t wf = 0;
  std::vector<const Node*> order;  // walk order of elements of this process

  void index_ids(const Node* n) {
    if (const char* id = n->get("id")) dom_ids[id] = n;
    for (auto& k : n->kids) index_ids(k.get());
  }

  // pre-order, children last-to-first (ModelWalker)
  void walk(const Node* n) {
    order.push_back(n);
    for (size_t i = n->kids.size(); i-- > 0;) walk(n->kids[i].get());
  }

  DevElem& E(uint16_t i) { return t.elems[i]; }

  uint16_t new_elem(uint8_t kind, const std::string& id) {
    DevElem e;
    memset(&e, 0, sizeof(e));
    e.kind = kind;
    e.wf = wf;
    memset(e.step, ST_UNBOUND, sizeof(e.step));
    e.out0 = e.target = e.start = e.dflt = NO_ELEM;
    e.cond_prog = NO_REF;
    e.headers_off = NO_REF;
    e.retries = 3;  // ZeebeTaskDefinition.DEFAULT_RETRIES
    e.id_off = t.add_bytes(id);
    e.id_len = (uint16_t)id.size();
    t.elems.push_back(e);
    t.elem_ids.push_back(id);
    uint16_t idx = (uint16_t)(t.elems.size() - 1);
    ids[id] = idx;  // later registrations of the same id win (HashMap.put)
    return idx;
  }

  // FlowNodeHandler (transformation/handler/FlowNodeHandler.java): zeebe:ioMapping inputs / outputs / output
  // behaviour, validated as ZeebeIoMappingValidator (broker-core/.../validation/ZeebeIoMappingValidator.java:36-57,
  // bpmn-model/.../validation/zeebe/ZeebeIoMappingValidator.java:31-39) and ZeebeExpressionValidator
  // (.validateJsonPath :42-54) validate them at deployment
  int io_mapping(DevElem& e, const Node* io) {
    std::vector<std::pair<std::string, std::string>> ins, outs;
    for (auto& k : io->kids) {
      if (k->tag != "input" && k->tag != "output") continue;
      const char* src = k->get("source");
      const char* tgt = k->get("target");
      (k->tag == "input" ? ins : outs).emplace_back(src ? src : "", tgt ? tgt : "");
    }
    uint8_t ob = OB_UNSET;
    if (const char* b = io->get("outputBehavior")) {
      const std::string bs(b);
      if (bs == "none") ob = OB_NONE;
      else if (bs == "merge") ob = OB_MERGE;
      else if (bs == "overwrite") ob = OB_OVERWRITE;
      else { err = "invalid outputBehavior: " + bs; return ZB_EDEPLOY; }
    }
    auto root_target = [](const std::vector<std::pair<std::string, std::string>>& ms) {
      for (auto& m : ms)
        if (m.second == "$") return true;
      return false;
    };
    if (ins.size() > 1 && root_target(ins)) { err = "Invalid inputs: When using $ as target, no other input can be defined"; return ZB_EDEPLOY; }
    if (outs.size() > 1 && root_target(outs)) { err = "Invalid outputs: When using $ as target, no other output can be defined"; return ZB_EDEPLOY; }
    if (ob == OB_NONE && !outs.empty()) {
      err = "Output behavior 'none' cannot be used in combination without zeebe:output elements";
      return ZB_EDEPLOY;
    }
    for (const auto* ms : {&ins, &outs})
      for (auto& m : *ms)
        for (const std::string& path : {m.first, m.second}) {
          ModelTables scratch;
          std::string qerr;
          if (compile_query(scratch, path, qerr) < 0) { err = "JSON path query is invalid: " + qerr; return ZB_EDEPLOY; }
          // PROHIBITED_PATHS_REGEX "(\\.\\*)|(\\[.*,.*\\])"
          const size_t lb = path.find('[');
          const size_t comma = lb == std::string::npos ? std::string::npos : path.find(',', lb + 1);
          if (path.find(".*") != std::string::npos ||
              (comma != std::string::npos && path.find(']', comma + 1) != std::string::npos)) {
            err = "This JSON path query is not supported";
            return ZB_EDEPLOY;
          }
        }
    if (ins.size() > 255 || outs.size() > 255) { err = "more than 255 io mappings on one element"; return ZB_EUNSUPPORTED; }
    e.flags |= EF_IO | (uint8_t)(ob << OB_SHIFT);
    e.map_in = (uint16_t)t.maps.size();
    e.n_in = (uint8_t)ins.size();
    for (auto& m : ins)
      if (compile_mapping(t, m.first, m.second, err) < 0) return ZB_EDEPLOY;
    e.map_out = (uint16_t)t.maps.size();
    e.n_out_map = (uint8_t)outs.size();
    for (auto& m : outs)
      if (compile_mapping(t, m.first, m.second, err) < 0) return ZB_EDEPLOY;
    if (t.maps.size() >= 0xffff) { err = "too many io mappings"; return ZB_EUNSUPPORTED; }
    return ZB_OK;
  }

  int process(const Node* proc, int64_t key, int32_t version) {
    ids.clear();
    order.clear();
    walk(proc);
    DevWorkflow w{};
    w.key = key;
    w.version = version;
    std::string pid = proc->get("id") ? proc->get("id") : "";
    w.pid_off = t.add_bytes(pid);
    w.pid_len = (uint16_t)pid.size();
    wf = (uint16_t)t.workflows.size();
    uint16_t pe = new_elem(EK_PROCESS, pid);
    w.process_elem = pe;
    t.workflows.push_back(w);
    DevElem& P = E(pe);
    P.step[WI_ELEMENT_READY] = ST_APPLY_INPUT_MAPPING;
    P.step[WI_ELEMENT_ACTIVATED] = ST_TRIGGER_START_EVENT;
    P.step[WI_ELEMENT_COMPLETING] = ST_COMPLETE_PROCESS;
    P.step[WI_ELEMENT_TERMINATING] = ST_TERMINATE_CONTAINED_INSTANCES;
    // pass 1: create elements (FlowElementHandler)
    for (const Node* n : order) {
      if (n == proc) continue;
      const std::string& g = n->tag;
      if (g != "sequenceFlow" && !is_flow_node_tag(g)) continue;
      uint8_t k;
      if (g == "startEvent") k = EK_START;
      else if (g == "endEvent") k = EK_END;
      else if (g == "serviceTask") k = EK_TASK;
      else if (g == "subProcess") k = EK_SUB;
      else if (g == "exclusiveGateway") k = EK_XOR;
      else if (g == "intermediateCatchEvent") k = EK_CATCH;
      else if (g == "sequenceFlow") k = EK_FLOW;
      else if (g == "parallelGateway") k = EK_PAR;  // EXTENSION (C4)
      else { err = "unsupported element type '" + g + "'"; return ZB_EUNSUPPORTED; }
      new_elem(k, n->get("id") ? n->get("id") : "");
    }
    // parallel gateways: join arity (sequence flows targeting the gateway) and, for joins, a counter slot
    // in the RowAux of their scope (the enclosing process / sub process)
    std::unordered_map<std::string, int> joins_in_scope;
    for (const Node* n : order) {
      if (n->tag != "sequenceFlow" || !n->get("targetRef")) continue;
      auto it = ids.find(n->get("targetRef"));
      if (it != ids.end() && E(it->second).kind == EK_PAR) {
        if (E(it->second).m_in == 255) { err = "parallel gateway with more than 254 incoming flows"; return ZB_EUNSUPPORTED; }
        E(it->second).m_in++;
      }
    }
    for (const Node* n : order) {
      if (n->tag != "parallelGateway") continue;
      DevElem& g = E(ids.at(n->get("id") ? n->get("id") : ""));
      if (g.m_in < 2) continue;
      const Node* sc = n->up;
      while (sc && sc->tag != "subProcess" && sc != proc) sc = sc->up;
      int& slot = joins_in_scope[sc && sc->get("id") ? sc->get("id") : ""];
      if (slot >= JOIN_SLOTS) { err = "more than 2 parallel joins directly inside one scope"; return ZB_EUNSUPPORTED; }
      g.join_slot = (uint8_t)slot++;
    }
    // pass 2: attributes, links, lifecycle bindings
    std::vector<std::vector<uint16_t>> outgoing(t.elems.size());
    std::vector<std::vector<uint16_t>> conditioned(t.elems.size());
    for (const Node* n : order) {
      if (n == proc) continue;
      const std::string& g = n->tag;
      if (g != "sequenceFlow" && !is_flow_node_tag(g)) continue;
      uint16_t ei = ids.at(n->get("id") ? n->get("id") : "");
      if (g == "sequenceFlow") {
        const char* s = n->get("sourceRef");
        const char* d = n->get("targetRef");
        if (!s || !d || !ids.count(s) || !ids.count(d)) { err = "sequence flow with unknown source/target"; return ZB_EDEPLOY; }
        uint16_t si = ids[s], di = ids[d];
        if (const Node* c = child(n, "conditionExpression")) {
          int prog = compile_condition(t, c->text, err);
          if (prog == -2) return ZB_EUNSUPPORTED;
          if (prog < 0) return ZB_EDEPLOY;
          E(ei).cond_prog = (uint32_t)prog;
        }
        outgoing[si].push_back(ei);
        if (E(si).kind == EK_XOR && E(ei).cond_prog != NO_REF) conditioned[si].push_back(ei);
        E(ei).target = di;
        uint8_t tk = E(di).kind;
        uint8_t st;
        if (tk == EK_TASK || tk == EK_SUB || tk == EK_CATCH) st = ST_START_STATEFUL_ELEMENT;
        else if (tk == EK_XOR) st = ST_ACTIVATE_GATEWAY;
        else if (tk == EK_END) st = ST_TRIGGER_END_EVENT;
        else if (tk == EK_PAR) st = E(di).m_in >= 2 ? ST_PARALLEL_MERGE : ST_ACTIVATE_GATEWAY;
        else { err = "Unsupported element"; return ZB_EUNSUPPORTED; }
        E(ei).step[WI_SEQUENCE_FLOW_TAKEN] = st;
        continue;
      }
      DevElem& e = E(ei);
      // FlowNodeHandler: io mapping + outgoing behaviour from <outgoing> references
      if (const Node* io = extension(n, "ioMapping")) {
        const int rc = io_mapping(e, io);
        if (rc != ZB_OK) return rc;
      }
      int n_out_refs = 0;
      for (auto& k : n->kids)
        if (k->tag == "outgoing") n_out_refs++;
      uint8_t outgoing_step = n_out_refs == 0 ? ST_CONSUME_TOKEN : ST_TAKE_SEQUENCE_FLOW;
      if (e.kind == EK_TASK || e.kind == EK_SUB) {  // ActivityHandler
        e.step[WI_ELEMENT_READY] = ST_APPLY_INPUT_MAPPING;
        e.step[WI_ELEMENT_COMPLETING] = ST_APPLY_OUTPUT_MAPPING;
        e.step[WI_ELEMENT_COMPLETED] = outgoing_step;
        e.step[WI_ELEMENT_TERMINATED] = ST_PROPAGATE_TERMINATION;
      }
      switch (e.kind) {
        case EK_END: e.step[WI_END_EVENT_OCCURRED] = outgoing_step; break;
        case EK_START: {
          const Node* scope = n->up;
          if (scope->tag == "subProcess") E(ids.at(scope->get("id"))).start = ei;
          else P_start(pe) = ei;
          e.step[WI_START_EVENT_OCCURRED] = outgoing_step;
          break;
        }
        case EK_XOR: {
          if (const char* d = n->get("default")) {
            if (ids.count(d)) e.dflt = ids[d];
          }
          bool first_cond = false;
          if (const Node* o = child(n, "outgoing")) {
            auto it = dom_ids.find(trim(o->text));
            first_cond = it != dom_ids.end() && child(it->second, "conditionExpression") != nullptr;
          }
          e.step[WI_GATEWAY_ACTIVATED] = first_cond ? ST_EXCLUSIVE_SPLIT : outgoing_step;
          break;
        }
        case EK_TASK: {
          if (const Node* td = extension(n, "taskDefinition")) {
            std::string ty = td->get("type") ? td->get("type") : "";
            e.type_off = t.add_bytes(ty);
            e.type_len = (uint16_t)ty.size();
            if (td->get("retries")) e.retries = atoi(td->get("retries"));
          }
          if (const Node* th = extension(n, "taskHeaders")) {  // ServiceTaskHandler.encode
            std::vector<std::pair<std::string, std::string>> hs;
            for (auto& k : th->kids)
              if (k->tag == "header")
                hs.emplace_back(k->get("key") ? k->get("key") : "", k->get("value") ? k->get("value") : "");
            std::string enc;
            if (!hs.empty()) {
              auto put_str = [&](const std::string& s) {
                size_t n2 = s.size();
                if (n2 < 32) enc += (char)(0xa0 | n2);
                else if (n2 < 256) { enc += (char)0xd9; enc += (char)n2; }
                else if (n2 < 65536) { enc += (char)0xda; enc += (char)(n2 >> 8); enc += (char)n2; }
                else { enc += (char)0xdb; for (int b = 3; b >= 0; b--) enc += (char)(n2 >> (8 * b)); }
                enc += s;
              };
              size_t m = hs.size();
              if (m < 16) enc += (char)(0x80 | m);
              else if (m < 65536) { enc += (char)0xde; enc += (char)(m >> 8); enc += (char)m; }
              else { enc += (char)0xdf; for (int b = 3; b >= 0; b--) enc += (char)(m >> (8 * b)); }
              for (auto& h : hs) { put_str(h.first); put_str(h.second); }
            }
            e.headers_off = t.add_bytes(enc);
            e.headers_len = (uint32_t)enc.size();
          }
          e.step[WI_ELEMENT_ACTIVATED] = ST_CREATE_JOB;
          e.step[WI_ELEMENT_TERMINATING] = ST_TERMINATE_JOB_TASK;
          break;
        }
        case EK_SUB:
          e.step[WI_ELEMENT_ACTIVATED] = ST_TRIGGER_START_EVENT;
          e.step[WI_ELEMENT_TERMINATING] = ST_TERMINATE_CONTAINED_INSTANCES;
          break;
        case EK_PAR:
          if (n_out_refs == 0) { err = "parallel gateway without outgoing sequence flow"; return ZB_EUNSUPPORTED; }
          e.step[WI_GATEWAY_ACTIVATED] = ST_PARALLEL_SPLIT;
          break;
        case EK_CATCH: {
          const Node* med = child(n, "messageEventDefinition");
          const char* mref = med ? med->get("messageRef") : nullptr;
          auto it = mref ? dom_ids.find(mref) : dom_ids.end();
          if (it == dom_ids.end()) { err = "intermediate catch event without message"; return ZB_EUNSUPPORTED; }
          const Node* msg = it->second;
          std::string name = msg->get("name") ? msg->get("name") : "";
          e.msg_off = t.add_bytes(name);
          e.msg_len = (uint16_t)name.size();
          const Node* sub = extension(msg, "subscription");
          std::string ck = sub && sub->get("correlationKey") ? sub->get("correlationKey") : "";
          int qi = compile_query(t, ck, err);
          if (qi < 0) return ZB_EDEPLOY;
          e.ck_query = (uint16_t)qi;
          e.step[WI_ELEMENT_READY] = ST_APPLY_INPUT_MAPPING;
          e.step[WI_ELEMENT_ACTIVATED] = ST_SUBSCRIBE_TO_INTERMEDIATE_MESSAGE;
          e.step[WI_ELEMENT_COMPLETING] = ST_APPLY_OUTPUT_MAPPING;
          e.step[WI_ELEMENT_COMPLETED] = outgoing_step;
          e.step[WI_ELEMENT_TERMINATING] = ST_TERMINATE_ELEMENT;
          e.step[WI_ELEMENT_TERMINATED] = ST_PROPAGATE_TERMINATION;
          break;
        }
      }
    }
    for (size_t i = 0; i < outgoing.size(); i++) {
      if (outgoing[i].empty() && conditioned[i].empty()) continue;
      DevElem& e = t.elems[i];
      e.n_out = (uint16_t)outgoing[i].size();
      if (!outgoing[i].empty()) e.out0 = outgoing[i][0];
      e.cond_begin = (uint16_t)t.cond_flows.size();
      e.cond_count = (uint16_t)conditioned[i].size();
      t.cond_flows.insert(t.cond_flows.end(), conditioned[i].begin(), conditioned[i].end());
      if (e.kind == EK_PAR) {  // fork: every outgoing flow, executable order
        if (outgoing[i].size() > (size_t)MAX_FANOUT) { err = "parallel gateway with more than 63 outgoing flows"; return ZB_EUNSUPPORTED; }
        e.out_begin = (uint16_t)t.cond_flows.size();
        t.cond_flows.insert(t.cond_flows.end(), outgoing[i].begin(), outgoing[i].end());
      }
    }
    if (t.cond_flows.size() >= 0xffff) { err = "too many sequence flows"; return ZB_EUNSUPPORTED; }
    return ZB_OK;
  }
  uint16_t& P_start(uint16_t pe) { return t.elems[pe].start; }
};

}  // namespace

int compile_query(ModelTables& t, const std::string& expr, std::string& err) {
  std::vector<DevFilter> fs;
  if (!compile_filters(expr, fs, t, err)) return -1;
  DevQuery q{};
  q.first = (uint16_t)t.filters.size();
  q.count = (uint16_t)fs.size();
  q.expr_off = t.add_bytes(expr);
  q.expr_len = (uint16_t)expr.size();
  q.fast = (fs.size() == 2 && fs[0].id == F_ROOT && fs[1].id == F_MAP_KEY) ? 1 : 0;
  t.filters.insert(t.filters.end(), fs.begin(), fs.end());
  t.queries.push_back(q);
  return (int)t.queries.size() - 1;
}

// JsonPathTokenizer (json-path/.../jsonpath/JsonPathTokenizer.java): operators in table order ("$", "..", ".",
// "*", "['", "']", "[", "]"), everything between them a LITERAL; after "['" only "']" is recognised
static void path_literals(const std::string& e, std::vector<std::pair<uint32_t, uint32_t>>& out) {
  static const char* OPS[8] = {"$", "..", ".", "*", "['", "']", "[", "]"};
  size_t pos = 0, last = 0;
  bool bracket = false;
  while (pos < e.size()) {
    bool hit = false;
    for (int i = 0; i < 8 && !hit; i++) {
      if (bracket && i != 5) continue;
      const size_t l = strlen(OPS[i]);
      if (e.compare(pos, l, OPS[i]) == 0) {
        if (last < pos) out.emplace_back((uint32_t)last, (uint32_t)(pos - last));
        if (i == 0) out.emplace_back((uint32_t)pos, 1u);  // ROOT_OBJECT
        bracket = i == 4;
        pos += l;
        last = pos;
        hit = true;
      }
    }
    if (!hit) pos++;
  }
  if (last < pos) out.emplace_back((uint32_t)last, (uint32_t)(pos - last));
}

int compile_mapping(ModelTables& t, const std::string& source, const std::string& target, std::string& err) {
  const int q = compile_query(t, source, err);
  if (q < 0) return -1;
  std::vector<std::pair<uint32_t, uint32_t>> lits;
  path_literals(target, lits);
  if (lits.empty() || lits.size() > 0xffff || t.maps.size() >= 0xffff) { err = "invalid mapping target"; return -1; }
  DevMapping m{};
  m.query = (uint16_t)q;
  m.nseg = (uint16_t)lits.size();
  m.seg = (uint32_t)t.segs.size();
  const uint32_t base = t.add_bytes(target);
  for (auto& l : lits) t.segs.push_back(DevSeg{base + l.first, l.second});
  t.maps.push_back(m);
  return (int)t.maps.size() - 1;
}

static bool has_large_int_const(const ModelTables& t, const CondAst* n) {
  if (n->op == 10 || n->op == 11) return has_large_int_const(t, n->l.get()) || has_large_int_const(t, n->r.get());
  auto big = [&](int is_path, int idx) {
    if (is_path) return false;
    const DevConst& c = t.consts[idx];
    return c.type == TT_INTEGER && (c.ival >= (1LL << 53) || c.ival <= -(1LL << 53));
  };
  return big(n->lhs_path, n->lhs) || big(n->rhs_path, n->rhs);
}

int compile_condition(ModelTables& t, const std::string& expr, std::string& err) {
  if (expr.empty()) { err = "expression is empty"; return -1; }
  CondParser p(expr, t);
  auto ast = p.parse(err);
  if (!ast) return -1;
  if (has_large_int_const(t, ast.get())) {
    // The reference promotes an INTEGER constant to FLOAT permanently once it meets a FLOAT
    // (JsonConditionInterpreter.ensureSameType :220-233). That history-dependent state only changes
    // results for |constant| >= 2^53, which the GPU path refuses rather than approximates.
    err = "integer constants with |value| >= 2^53 are not supported by the GPU condition VM";
    return -2;
  }
  int off = (int)t.code.size();
  emit(t, ast.get());
  t.code.push_back(PC_END);
  t.code.push_back(0);
  return off / 2;  // instruction index
}

int compile_deployment(ModelTables& t, const std::string& xml, int64_t workflow_key, int32_t version,
                       std::string& err) {
  std::unique_ptr<Node> doc;
  try {
    doc = parse_xml(xml);
  } catch (const XmlError& e) {
    err = "xml: " + e.msg;
    return ZB_EDEPLOY;
  }
  const Node* defs = child(doc.get(), "definitions");
  if (!defs) { err = "no bpmn definitions"; return ZB_EDEPLOY; }
  ModelTables backup = t;  // all-or-nothing
  Deployer d{t, err};
  d.index_ids(defs);
  int64_t k = workflow_key;
  int rc = ZB_OK;
  for (auto& c : defs->kids) {
    if (c->tag != "process") continue;
    rc = d.process(c.get(), k++, version);
    if (rc != ZB_OK) break;
  }
  if (rc == ZB_OK && t.elems.size() >= NO_ELEM) { err = "too many elements"; rc = ZB_EUNSUPPORTED; }
  if (rc != ZB_OK) t = backup;
  return rc;
}

}  // namespace zbg
