// ORACLE / TEST INFRASTRUCTURE ONLY. Never linked into the product (zeebe_amd/csrc).
//
// json-el conditions restated from the reference:
//   grammar:      json-el/src/main/scala/io/zeebe/msgpack/el/JsonConditionParser.scala:37-114
//                 (scala-parser-combinators 1.0.6 JavaTokenParsers; whitespace skipped before every
//                 literal/regex; `~!` commits; phrase() reports the deepest recorded failure)
//   factory:      json-el/src/main/java/io/zeebe/msgpack/el/JsonConditionFactory.java:26-76
//   validator:    json-el/src/main/java/io/zeebe/msgpack/el/JsonConditionValidator.java
//   interpreter:  json-el/src/main/java/io/zeebe/msgpack/el/JsonConditionInterpreter.java:38-240
// Constants are mutable tokens owned by the AST, exactly like the Scala case objects: an INTEGER
// constant compared against a FLOAT is promoted to FLOAT *permanently* (ensureSameType :220-233).
#pragma once
#include <cmath>
#include <cstdlib>
#include <memory>
#include <cctype>
#include <string>
#include <vector>

#include "zbref_jsonpath.hpp"

namespace zbref {

struct ConditionError : std::runtime_error {  // JsonConditionException
  using std::runtime_error::runtime_error;
};

struct ElObject {
  bool is_path = false;
  JsonPathQuery query;  // for paths
  MpToken token;        // for constants (mutable!)
  bytes str_storage;    // backing storage for string constants
};

enum class ElOp { EQ, NE, LT, LE, GT, GE, AND, OR };

struct ElNode {
  ElOp op;
  std::unique_ptr<ElObject> x, y;      // comparisons
  std::unique_ptr<ElNode> l, r;        // operators
};

struct CompiledCondition {
  std::string expression;
  std::unique_ptr<ElNode> root;
  bool valid = false;
  std::string error;
};

// ------------------------------------------------------------------------------------- parser
class ElParser {
 public:
  explicit ElParser(const std::string& in) : s(in) {}

  // parseAll(condition, in)
  std::unique_ptr<ElNode> parse_all(std::string& err) {
    last_pos = -1;
    size_t pos = 0;
    std::unique_ptr<ElNode> n;
    Res r = condition(pos, n);
    if (r == OK) {
      size_t p = skip_ws(pos);
      if (p == s.size()) return n;
      if (last_pos >= 0 && (size_t)last_pos >= pos) { err = format(last_msg, (size_t)last_pos); return nullptr; }
      err = format("end of input expected", pos);
      return nullptr;
    }
    err = format(last_msg, (size_t)(last_pos < 0 ? 0 : last_pos));
    return nullptr;
  }

 private:
  enum Res { OK, FAIL, ERR };
  const std::string& s;
  long last_pos = -1;
  std::string last_msg;

  // NoSuccess constructor side effect: remember the deepest (ties: latest) failure.
  void record(const std::string& msg, size_t pos) {
    if (last_pos < 0 || !((long)pos < last_pos)) { last_pos = (long)pos; last_msg = msg; }
  }
  std::string format(const std::string& msg, size_t pos) {
    // ParseResult.toString: "[line.col] failure: msg\n\n<line>\n<caret>"
    std::string out = "[1." + std::to_string(pos + 1) + "] failure: " + msg + "\n\n" + s + "\n";
    out += std::string(pos, ' ') + "^";
    return out;
  }
  size_t skip_ws(size_t p) const {
    while (p < s.size() && (s[p] == ' ' || s[p] == '\t' || s[p] == '\n' || s[p] == '\r' || s[p] == '\f' ||
                            s[p] == '\x0b'))
      p++;
    return p;
  }
  std::string found(size_t p) const {
    if (p >= s.size()) return "end of source";
    return std::string("`") + s[p] + "'";
  }
  // literal("xx") parser
  bool lit(size_t& pos, const char* l) {
    size_t p = skip_ws(pos);
    size_t n = std::strlen(l);
    if (s.compare(p, n, l) == 0) { pos = p + n; return true; }
    record(std::string("`") + l + "' expected but " + found(p) + " found", p);
    fail_pos = p;
    return false;
  }
  size_t fail_pos = 0;  // position of the failure returned by the last failing primitive

  // ---- regex primitives ----
  bool json_path(size_t& pos, bytes& out) {  // \$([^\s])*
    size_t p = skip_ws(pos);
    if (p < s.size() && s[p] == '$') {
      size_t e = p + 1;
      while (e < s.size() && !(s[e] == ' ' || s[e] == '\t' || s[e] == '\n' || s[e] == '\r' || s[e] == '\f' ||
                               s[e] == '\x0b'))
        e++;
      out = s.substr(p, e - p);
      pos = e;
      return true;
    }
    record("string matching regex `\\$([^\\s])*' expected but " + found(p) + " found", p);
    fail_pos = p;
    return false;
  }
  static bool is_digit(char c) { return c >= '0' && c <= '9'; }
  // number: -?(\d+\.\d*|\d*\.\d+)([eE][+-]?\d+)?[fFdD]?  => double ; else -?\d+ => long
  bool number(size_t& pos, MpToken& tok) {
    size_t p = skip_ws(pos);
    size_t i = p;
    if (i < s.size() && s[i] == '-') i++;
    size_t d0 = i;
    while (i < s.size() && is_digit(s[i])) i++;
    size_t nint = i - d0;
    bool is_float = false;
    size_t e = i;
    if (i < s.size() && s[i] == '.') {
      size_t j = i + 1;
      while (j < s.size() && is_digit(s[j])) j++;
      size_t nfrac = j - (i + 1);
      if (nint > 0 || nfrac > 0) {
        is_float = true;
        e = j;
        if (e < s.size() && (s[e] == 'e' || s[e] == 'E')) {
          size_t k = e + 1;
          if (k < s.size() && (s[k] == '+' || s[k] == '-')) k++;
          size_t k0 = k;
          while (k < s.size() && is_digit(s[k])) k++;
          if (k > k0) e = k;
        }
        if (e < s.size() && (s[e] == 'f' || s[e] == 'F' || s[e] == 'd' || s[e] == 'D')) e++;
      }
    }
    if (is_float) {
      std::string t = s.substr(p, e - p);
      if (!t.empty() && (t.back() == 'f' || t.back() == 'F' || t.back() == 'd' || t.back() == 'D')) t.pop_back();
      tok = MpToken();
      tok.type = MpType::FLOAT;
      tok.fval = std::strtod(t.c_str(), nullptr);  // Java Double.parseDouble (round-to-nearest)
      pos = e;
      return true;
    }
    if (nint > 0) {
      tok = MpToken();
      tok.type = MpType::INTEGER;
      tok.ival = std::strtoll(s.substr(p, i - p).c_str(), nullptr, 10);
      pos = i;
      return true;
    }
    record("string matching regex `-?\\d+' expected but " + found(p) + " found", p);
    fail_pos = p;
    return false;
  }
  bool hex4(size_t i) const {  // \\u[a-fA-F0-9]{4}
    for (size_t k = i; k < i + 4; k++)
      if (k >= s.size() || !std::isxdigit((unsigned char)s[k])) return false;
    return true;
  }
  // string: JavaTokenParsers.stringLiteral (kept raw, no unescaping) | '...'
  bool string_lit(size_t& pos, bytes& out) {
    size_t p = skip_ws(pos);
    if (p < s.size() && s[p] == '"') {
      size_t i = p + 1;
      bool ok = false;
      while (i < s.size()) {
        unsigned char c = (unsigned char)s[i];
        if (c == '"') { ok = true; break; }
        if (c == '\\') {
          if (i + 1 < s.size() && std::strchr("\\'\"bfnrt", s[i + 1])) { i += 2; continue; }
          if (i + 5 < s.size() && s[i + 1] == 'u' && hex4(i + 2)) { i += 6; continue; }
          break;
        }
        if (c < 0x20 || c == 0x7f) break;
        i++;
      }
      if (ok) { out = s.substr(p + 1, i - p - 1); pos = i + 1; return true; }
      record("string matching regex `\"...\"' expected but " + found(p) + " found", p);
      fail_pos = p;
      // fall through to the single-quote alternative
    }
    if (p < s.size() && s[p] == '\'') {
      size_t i = p + 1;
      while (i < s.size()) {
        unsigned char c = (unsigned char)s[i];
        if (c == '\'' || c == '"' || c < 0x20 || c == 0x7f) break;
        if (c == '\\') {
          if (i + 1 < s.size() && std::strchr("\\'\"bfnrt", s[i + 1])) { i += 2; continue; }
          if (i + 5 < s.size() && s[i + 1] == 'u' && hex4(i + 2)) { i += 6; continue; }
          break;
        }
        i++;
      }
      if (i < s.size() && s[i] == '\'') { out = s.substr(p + 1, i - p - 1); pos = i + 1; return true; }
      record(std::string("`'' expected but ") + found(i) + " found", i);
      fail_pos = i;
      return false;
    }
    record("string matching regex `\"...\"' expected but " + found(p) + " found", p);
    fail_pos = p;
    return false;
  }

  std::unique_ptr<ElObject> make_path(const bytes& text) {
    auto o = std::make_unique<ElObject>();
    o->is_path = true;
    JsonPathCompiler c;
    o->query = c.compile(text);
    return o;
  }

  // literal = jsonPath | string | number | true | false | null   withFailureMessage(...)
  Res literal(size_t& pos, std::unique_ptr<ElObject>& out) {
    size_t p = pos;
    size_t furthest = 0;
    bytes b;
    if (json_path(p, b)) { out = make_path(b); pos = p; return OK; }
    furthest = std::max(furthest, fail_pos);
    p = pos;
    if (string_lit(p, b)) {
      out = std::make_unique<ElObject>();
      out->str_storage = b;
      out->token.type = MpType::STRING;
      out->token.data = (const uint8_t*)out->str_storage.data();
      out->token.len = (uint32_t)out->str_storage.size();
      pos = p;
      return OK;
    }
    furthest = std::max(furthest, fail_pos);
    p = pos;
    MpToken t;
    if (number(p, t)) { out = std::make_unique<ElObject>(); out->token = t; pos = p; return OK; }
    furthest = std::max(furthest, fail_pos);
    const char* kw[3] = {"true", "false", "null"};
    for (int k = 0; k < 3; k++) {
      p = pos;
      if (lit(p, kw[k])) {
        out = std::make_unique<ElObject>();
        if (k == 2) out->token.type = MpType::NIL;
        else { out->token.type = MpType::BOOLEAN; out->token.bval = k == 0; }
        pos = p;
        return OK;
      }
      furthest = std::max(furthest, fail_pos);
    }
    record("expected literal (JSON path, string, number, boolean, null)", furthest);
    fail_pos = furthest;
    return FAIL;
  }

  Res number_or_path(size_t& pos, std::unique_ptr<ElObject>& out) {
    size_t p = pos, furthest = 0;
    MpToken t;
    if (number(p, t)) { out = std::make_unique<ElObject>(); out->token = t; pos = p; return OK; }
    furthest = std::max(furthest, fail_pos);
    p = pos;
    bytes b;
    if (json_path(p, b)) { out = make_path(b); pos = p; return OK; }
    furthest = std::max(furthest, fail_pos);
    record("expected number or JSON path", furthest);
    fail_pos = furthest;
    return FAIL;
  }

  // commit(): a Failure becomes an Error (recorded again at the same position)
  Res commit(Res r) {
    if (r == FAIL) { record(last_msg_at(fail_pos), fail_pos); return ERR; }
    return r;
  }
  std::string last_msg_at(size_t) const { return last_msg; }

  Res comparison(size_t& pos, std::unique_ptr<ElNode>& out) {
    size_t furthest = 0;
    // alt 1: literal ~ ("==" | "!=") ~! literal
    {
      size_t p = pos;
      std::unique_ptr<ElObject> x;
      Res r = literal(p, x);
      if (r == OK) {
        size_t q = p;
        ElOp op;
        bool m = false;
        if (lit(q, "==")) { op = ElOp::EQ; m = true; }
        else {
          size_t f1 = fail_pos;
          q = p;
          if (lit(q, "!=")) { op = ElOp::NE; m = true; }
          else fail_pos = std::max(f1, fail_pos);
        }
        if (m) {
          std::unique_ptr<ElObject> y;
          Res r2 = commit(literal(q, y));
          if (r2 != OK) return ERR;
          out = std::make_unique<ElNode>();
          out->op = op; out->x = std::move(x); out->y = std::move(y);
          pos = q;
          return OK;
        }
      }
      furthest = std::max(furthest, fail_pos);
    }
    // alt 2: (number | jsonPath) ~ ("<=" | ">=" | "<" | ">") ~! numberOrJsonPath
    {
      size_t p = pos;
      std::unique_ptr<ElObject> x;
      Res r = number_or_path(p, x);
      if (r == OK) {
        static const struct { const char* t; ElOp op; } OPS[4] = {
            {"<=", ElOp::LE}, {">=", ElOp::GE}, {"<", ElOp::LT}, {">", ElOp::GT}};
        size_t fp = 0;
        for (int k = 0; k < 4; k++) {
          size_t q = p;
          if (lit(q, OPS[k].t)) {
            std::unique_ptr<ElObject> y;
            Res r2 = commit(number_or_path(q, y));
            if (r2 != OK) return ERR;
            out = std::make_unique<ElNode>();
            out->op = OPS[k].op; out->x = std::move(x); out->y = std::move(y);
            pos = q;
            return OK;
          }
          fp = std::max(fp, fail_pos);
        }
        fail_pos = fp;
      }
      furthest = std::max(furthest, fail_pos);
    }
    // alt 3: "(" ~! condition ~ ")"
    {
      size_t p = pos;
      if (lit(p, "(")) {
        std::unique_ptr<ElNode> c;
        Res r = condition(p, c);
        if (r == ERR) return ERR;
        if (r == FAIL) { commit(FAIL); return ERR; }
        if (!lit(p, ")")) { commit(FAIL); return ERR; }
        out = std::move(c);
        pos = p;
        return OK;
      }
      furthest = std::max(furthest, fail_pos);
    }
    record("expected comparison operator ('==', '!=', '<', '<=', '>', '>=')", furthest);
    fail_pos = furthest;
    return FAIL;
  }

  // conjunction = chainl1(comparison | failure("expected comparison"), "&&" ^^^ Conjunction)
  Res comparison_or_fail(size_t& pos, std::unique_ptr<ElNode>& out) {
    Res r = comparison(pos, out);
    if (r != FAIL) return r;
    size_t f = fail_pos;
    record("expected comparison", pos);  // failure() does not skip whitespace
    fail_pos = std::max(f, pos) == f ? f : pos;
    // `|` returns the further of the two failures (tie: the latter)
    fail_pos = (f > pos) ? f : pos;
    return FAIL;
  }
  Res conjunction(size_t& pos, std::unique_ptr<ElNode>& out) {
    Res r = comparison_or_fail(pos, out);
    if (r != OK) return r;
    while (true) {
      size_t p = pos;
      if (!lit(p, "&&")) break;
      std::unique_ptr<ElNode> rhs;
      Res r2 = comparison_or_fail(p, rhs);
      if (r2 == ERR) return ERR;
      if (r2 == FAIL) break;
      auto n = std::make_unique<ElNode>();
      n->op = ElOp::AND; n->l = std::move(out); n->r = std::move(rhs);
      out = std::move(n);
      pos = p;
    }
    return OK;
  }
  Res disjunction(size_t& pos, std::unique_ptr<ElNode>& out) {
    Res r = conjunction(pos, out);
    if (r != OK) return r;
    while (true) {
      size_t p = pos;
      if (!lit(p, "||")) break;
      std::unique_ptr<ElNode> rhs;
      Res r2 = conjunction(p, rhs);
      if (r2 == ERR) return ERR;
      if (r2 == FAIL) break;
      auto n = std::make_unique<ElNode>();
      n->op = ElOp::OR; n->l = std::move(out); n->r = std::move(rhs);
      out = std::move(n);
      pos = p;
    }
    return OK;
  }
  Res condition(size_t& pos, std::unique_ptr<ElNode>& out) {
    Res r = disjunction(pos, out);
    if (r != FAIL) return r;
    record("expected comparison, disjunction or conjunction.", pos);
    fail_pos = pos;
    return FAIL;
  }
};

inline void el_walk_paths(ElNode* n, std::vector<ElObject*>& out) {
  if (n->op == ElOp::AND || n->op == ElOp::OR) {
    el_walk_paths(n->l.get(), out);
    el_walk_paths(n->r.get(), out);
  } else {
    if (n->x->is_path) out.push_back(n->x.get());
    if (n->y->is_path) out.push_back(n->y.get());
  }
}

// JsonConditionFactory.createCondition
inline CompiledCondition create_condition(const std::string& expr) {
  CompiledCondition c;
  c.expression = expr;
  if (expr.empty()) { c.error = "expression is empty"; return c; }
  ElParser p(expr);
  std::string err;
  auto root = p.parse_all(err);
  if (!root) { c.error = err; return c; }
  std::vector<ElObject*> paths;
  el_walk_paths(root.get(), paths);
  std::string verr;
  for (auto* o : paths) {
    if (!o->query.valid()) {
      if (!verr.empty()) verr += "\n";
      verr += o->query.error;
    }
  }
  if (!verr.empty()) { c.error = verr; return c; }
  c.root = std::move(root);
  c.valid = true;
  return c;
}

// ------------------------------------------------------------------------------------- interpreter
class ElInterpreter {
 public:
  bool eval(ElNode* c, const uint8_t* doc, size_t n) { return eval_condition(c, doc, n); }

 private:
  JsonPathExecutor exec;
  MpToken tx, ty;  // reader tokens (msgPackReader1 / msgPackReader2)

  bool eval_condition(ElNode* c, const uint8_t* doc, size_t n) {
    switch (c->op) {
      case ElOp::OR: return eval_condition(c->l.get(), doc, n) || eval_condition(c->r.get(), doc, n);
      case ElOp::AND: return eval_condition(c->l.get(), doc, n) && eval_condition(c->r.get(), doc, n);
      default: return eval_comparison(c, doc, n);
    }
  }
  MpToken* get_token(ElObject* o, const uint8_t* doc, size_t n, MpToken& reader_tok) {
    if (!o->is_path) return &o->token;
    exec.run(o->query.filters, doc, n);
    if (exec.results.empty())
      throw ConditionError("JSON path '" + o->query.expression + "' has no result.");
    if (exec.results.size() > 1)
      throw ConditionError("JSON path '" + o->query.expression + "' has more than one result.");
    MpReader r(doc + exec.results[0].position, (size_t)exec.results[0].length);
    reader_tok = r.read_token();
    return &reader_tok;
  }
  bool eval_comparison(ElNode* c, const uint8_t* doc, size_t n) {
    MpToken* x = get_token(c->x.get(), doc, n, tx);
    MpToken* y = get_token(c->y.get(), doc, n, ty);
    switch (c->op) {
      case ElOp::EQ: return equals(x, y);
      case ElOp::NE: return !equals(x, y);
      case ElOp::LT: same_type(x, y); ensure_number(x);
        return x->type == MpType::INTEGER ? x->ival < y->ival : x->fval < y->fval;
      case ElOp::LE: same_type(x, y); ensure_number(x);
        return x->type == MpType::INTEGER ? x->ival <= y->ival : x->fval <= y->fval;
      case ElOp::GT: same_type(x, y); ensure_number(x);
        return x->type == MpType::INTEGER ? x->ival > y->ival : x->fval > y->fval;
      case ElOp::GE: same_type(x, y); ensure_number(x);
        return x->type == MpType::INTEGER ? x->ival >= y->ival : x->fval >= y->fval;
      default: throw ZbError("Illegal comparison");
    }
  }
  static bool equals(MpToken* x, MpToken* y) {
    if (x->type == MpType::NIL) return y->type == MpType::NIL;
    if (y->type == MpType::NIL) return false;
    same_type(x, y);
    switch (x->type) {
      case MpType::STRING: return x->len == y->len && std::memcmp(x->data, y->data, x->len) == 0;
      case MpType::BOOLEAN: return x->bval == y->bval;
      case MpType::INTEGER: return x->ival == y->ival;
      case MpType::FLOAT: return x->fval == y->fval;
      default: throw ConditionError(std::string("Cannot compare value of type: ") + mp_type_name(x->type));
    }
  }
  static void same_type(MpToken* x, MpToken* y) {
    if (x->type == MpType::INTEGER && y->type == MpType::FLOAT) {
      x->type = MpType::FLOAT; x->fval = (double)x->ival;
    } else if (x->type == MpType::FLOAT && y->type == MpType::INTEGER) {
      y->type = MpType::FLOAT; y->fval = (double)y->ival;
    } else if (x->type != y->type) {
      throw ConditionError(std::string("Cannot compare values of different types: ") + mp_type_name(x->type) +
                           " and " + mp_type_name(y->type));
    }
  }
  static void ensure_number(MpToken* x) {
    if (x->type != MpType::INTEGER && x->type != MpType::FLOAT)
      throw ConditionError(std::string("Cannot compare values. Expected number but found: ") +
                           mp_type_name(x->type));
  }
};

}  // namespace zbref
