// ORACLE / TEST INFRASTRUCTURE ONLY. Never linked into the product (zeebe_amd/csrc).
//
// json-path compile + streaming query over msgpack, restated from the reference:
//   tokenizer: json-path/src/main/java/io/zeebe/msgpack/jsonpath/JsonPathTokenizer.java:59-106
//   compiler:  json-path/src/main/java/io/zeebe/msgpack/jsonpath/JsonPathQueryCompiler.java:51-125
//   executor:  json-path/src/main/java/io/zeebe/msgpack/query/MsgPackQueryExecutor.java:60-144
//   filters:   json-path/src/main/java/io/zeebe/msgpack/filter/*.java
//   traverser: json-path/src/main/java/io/zeebe/msgpack/query/MsgPackTraverser.java:47-64
// The executor is the reference's exact state machine (including its quirk that a scalar match of
// a non-final filter advances the *parent* level's filter, so `$.a.b` matches `{"a":1,"b":2}`).
#pragma once
#include <string>
#include <vector>

#include "zbref_msgpack.hpp"

namespace zbref {

enum JpFilterId { JP_ROOT = 0, JP_MAP_KEY = 1, JP_INDEX = 2, JP_WILDCARD = 3 };

struct JpFilter {
  int id;
  int32_t index = 0;
  bytes key;
};

enum class JpToken { START_INPUT, END_INPUT, ROOT_OBJECT, CHILD_OPERATOR, RECURSION_OPERATOR, WILDCARD,
                     SUBSCRIPT_OPERATOR_BEGIN, SUBSCRIPT_OPERATOR_END, CHILD_BRACKET_OPERATOR_BEGIN,
                     CHILD_BRACKET_OPERATOR_END, LITERAL };

inline const char* jp_token_name(JpToken t) {
  switch (t) {
    case JpToken::START_INPUT: return "START_INPUT";
    case JpToken::END_INPUT: return "END_INPUT";
    case JpToken::ROOT_OBJECT: return "ROOT_OBJECT";
    case JpToken::CHILD_OPERATOR: return "CHILD_OPERATOR";
    case JpToken::RECURSION_OPERATOR: return "RECURSION_OPERATOR";
    case JpToken::WILDCARD: return "WILDCARD";
    case JpToken::SUBSCRIPT_OPERATOR_BEGIN: return "SUBSCRIPT_OPERATOR_BEGIN";
    case JpToken::SUBSCRIPT_OPERATOR_END: return "SUBSCRIPT_OPERATOR_END";
    case JpToken::CHILD_BRACKET_OPERATOR_BEGIN: return "CHILD_BRACKET_OPERATOR_BEGIN";
    case JpToken::CHILD_BRACKET_OPERATOR_END: return "CHILD_BRACKET_OPERATOR_END";
    default: return "LITERAL";
  }
}

// JsonPathTokenizer.tokenize (json-path/.../jsonpath/JsonPathTokenizer.java:67-116): static tokens matched in
// table order, everything between them a LITERAL; after "['" only "']" is recognised.
template <class F>
inline void jp_tokenize(const bytes& expr, F&& visit) {
  static const struct { JpToken t; const char* rep; } ALL[8] = {
      {JpToken::ROOT_OBJECT, "$"}, {JpToken::RECURSION_OPERATOR, ".."}, {JpToken::CHILD_OPERATOR, "."},
      {JpToken::WILDCARD, "*"}, {JpToken::CHILD_BRACKET_OPERATOR_BEGIN, "['"},
      {JpToken::CHILD_BRACKET_OPERATOR_END, "']"}, {JpToken::SUBSCRIPT_OPERATOR_BEGIN, "["},
      {JpToken::SUBSCRIPT_OPERATOR_END, "]"}};
  const int length = (int)expr.size();
  int position = 0, last_end = 0;
  bool child_bracket = false;
  visit(JpToken::START_INPUT, 0, length);
  while (position < length) {
    bool matched = false;
    for (int i = 0; i < 8 && !matched; i++) {
      if (child_bracket && ALL[i].t != JpToken::CHILD_BRACKET_OPERATOR_END) continue;
      const size_t rl = std::strlen(ALL[i].rep);
      if (position + rl <= expr.size() && expr.compare(position, rl, ALL[i].rep) == 0) {
        if (last_end < position) visit(JpToken::LITERAL, last_end, position - last_end);
        child_bracket = ALL[i].t == JpToken::CHILD_BRACKET_OPERATOR_BEGIN;
        visit(ALL[i].t, position, (int)rl);
        position += (int)rl;
        last_end = position;
        matched = true;
      }
    }
    if (!matched) position++;
  }
  if (last_end < position) visit(JpToken::LITERAL, last_end, position - last_end);
  visit(JpToken::END_INPUT, 0, length);
}

struct JsonPathQuery {
  bytes expression;
  std::vector<JpFilter> filters;
  int invalid_position = -1;
  std::string error;
  bool valid() const { return invalid_position == -1; }
};

struct JsonPathCompiler {
  enum Mode { DEFAULT, SUBORDINATE } mode = DEFAULT;
  JsonPathQuery* q = nullptr;

  void visit(JpToken type, const bytes& expr, int off, int len) {
    if (!q->valid()) return;
    if (mode == DEFAULT) {
      switch (type) {
        case JpToken::ROOT_OBJECT: q->filters.push_back({JP_ROOT}); return;
        case JpToken::CHILD_OPERATOR:
        case JpToken::SUBSCRIPT_OPERATOR_BEGIN:
        case JpToken::CHILD_BRACKET_OPERATOR_BEGIN: mode = SUBORDINATE; return;
        case JpToken::START_INPUT:
        case JpToken::END_INPUT:
        case JpToken::SUBSCRIPT_OPERATOR_END:
        case JpToken::CHILD_BRACKET_OPERATOR_END: return;
        default:
          q->invalid_position = off;
          q->error = std::string("Unexpected json-path token ") + jp_token_name(type);
      }
    } else {
      switch (type) {
        case JpToken::LITERAL: {
          bool numeric = true;  // ByteUtil.isNumeric (json-path/.../util/ByteUtil.java:67-76)
          for (int i = off; i < off + len; i++) {
            int8_t c = (int8_t)expr[i];
            if (c < 48 || c > 57) { numeric = false; break; }
          }
          if (numeric) {
            int32_t v = 0, e = 1;  // ByteUtil.parseInteger :82-92 (int wraparound)
            for (int i = len - 1; i >= 0; i--) {
              v = (int32_t)((uint32_t)v + (uint32_t)((expr[off + i] - 48) * e));
              e = (int32_t)((uint32_t)e * 10u);
            }
            JpFilter f{JP_INDEX}; f.index = v; q->filters.push_back(f);
          } else {
            JpFilter f{JP_MAP_KEY}; f.key = expr.substr(off, len); q->filters.push_back(f);
          }
          mode = DEFAULT;
          return;
        }
        case JpToken::START_INPUT:
        case JpToken::END_INPUT: return;
        case JpToken::WILDCARD: q->filters.push_back({JP_WILDCARD}); return;
        default:
          q->invalid_position = off;
          q->error = std::string("Unexpected json-path token ") + jp_token_name(type);
      }
    }
  }

  JsonPathQuery compile(const bytes& expr) {
    JsonPathQuery query;
    query.expression = expr;
    q = &query;
    mode = DEFAULT;
    jp_tokenize(expr, [&](JpToken t, int off, int len) { visit(t, expr, off, len); });
    q = nullptr;
    return query;
  }
};

struct JpResult {
  int position;
  int length;
};

// MsgPackQueryExecutor + MsgPackTraverser
struct JsonPathExecutor {
  struct Level {
    int current = 0, num = 0, applying = 0;
    bool is_map = true;  // container type 0 == map; zero-initialised element => map
    int dyn = 0;
  };
  const std::vector<JpFilter>* filters = nullptr;
  std::vector<Level> ctx;
  std::vector<JpResult> results;
  int matching_container = -1;
  int matching_container_start = 0;

  bool filter_matches(const JpFilter& f, const MpToken& v) {
    switch (f.id) {
      case JP_ROOT: return ctx.empty() && mp_is_scalar(v.type) == false;
      case JP_MAP_KEY: {
        if (!ctx.empty() && ctx.back().is_map) {
          Level& l = ctx.back();
          if (l.current == 0) l.dyn = -1;
          int matching = l.dyn;
          if (l.current == matching) { l.dyn = -1; return true; }
          if (l.current % 2 == 0 && v.type == MpType::STRING && v.len == f.key.size() &&
              std::memcmp(v.data, f.key.data(), v.len) == 0) {
            l.dyn = l.current + 1;
          }
        }
        return false;
      }
      case JP_INDEX: return !ctx.empty() && !ctx.back().is_map && f.index == ctx.back().current;
      case JP_WILDCARD:
        if (!ctx.empty() && ctx.back().is_map) return ctx.back().current % 2 != 0;
        return true;
    }
    return false;
  }

  void visit(int position, const MpToken& v) {
    int current_filter = 0;
    if (!ctx.empty()) {
      ctx.back().current += 1;
      current_filter = ctx.back().applying;
    }
    bool match = false;
    if (current_filter >= 0) match = filter_matches((*filters)[current_filter], v);
    if (v.type == MpType::ARRAY || v.type == MpType::MAP) {
      Level l;
      l.current = -1;
      l.num = v.type == MpType::MAP ? (int)v.size * 2 : (int)v.size;
      l.applying = -1;
      l.is_map = v.type == MpType::MAP;
      ctx.push_back(l);
    }
    if (match) {
      if (current_filter + 1 == (int)filters->size()) {
        if (mp_is_scalar(v.type)) results.push_back({position, (int)v.total});
        else { matching_container = (int)ctx.size() - 1; matching_container_start = position; }
      } else {
        ctx.back().applying = current_filter + 1;
      }
    }
    while (!ctx.empty() && ctx.back().current + 1 >= ctx.back().num) {
      if (matching_container == (int)ctx.size() - 1) {
        results.push_back({matching_container_start, position + (int)v.total - matching_container_start});
        matching_container = -1;
      }
      ctx.pop_back();
    }
  }

  // MsgPackQueryProcessor.process: traverse the whole document (no early exit)
  void run(const std::vector<JpFilter>& f, const uint8_t* doc, size_t n) {
    filters = &f;
    ctx.clear();
    results.clear();
    matching_container = -1;
    if (f.empty()) return;
    MpReader r(doc, n);
    while (r.has_next()) {
      int pos = (int)r.off;
      MpToken t;
      try {
        t = r.read_token();
      } catch (const ZbError&) {
        return;  // traverser stops on an invalid token
      }
      visit(pos, t);
    }
  }
};

}  // namespace zbref
