// ORACLE / TEST INFRASTRUCTURE ONLY. Never linked into the product (zeebe_amd/csrc).
//
// Minimal XML reader for BPMN deployment resources (the oracle's own; the product has a separate
// reader in zeebe_amd/csrc). Element and attribute names are reduced to their local names, which
// is how the reference's camunda-xml-model 7.9.0 matches BPMN/zeebe elements by namespace+name.
#pragma once
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "zbref_msgpack.hpp"

namespace zbref {

struct XmlNode {
  std::string name;  // local name
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<XmlNode>> children;
  std::string text;  // concatenated character data (getTextContent of a leaf element)
  XmlNode* parent = nullptr;
  const std::string* attr(const std::string& k) const {
    for (auto& a : attrs)
      if (a.first == k) return &a.second;
    return nullptr;
  }
};

class XmlReader {
 public:
  std::unique_ptr<XmlNode> parse(const std::string& src) {
    s = &src;
    p = 0;
    auto root = std::make_unique<XmlNode>();
    root->name = "#document";
    std::vector<XmlNode*> stack{root.get()};
    while (p < s->size()) {
      if ((*s)[p] == '<') {
        if (starts("<?")) { skip_to("?>"); continue; }
        if (starts("<!--")) { skip_to("-->"); continue; }
        if (starts("<![CDATA[")) {
          size_t e = s->find("]]>", p + 9);
          if (e == std::string::npos) throw ZbError("unterminated CDATA");
          stack.back()->text += s->substr(p + 9, e - p - 9);
          p = e + 3;
          continue;
        }
        if (starts("<!")) { skip_to(">"); continue; }
        if (starts("</")) {
          size_t e = s->find('>', p);
          if (e == std::string::npos) throw ZbError("unterminated end tag");
          if (stack.size() <= 1) throw ZbError("unbalanced end tag");
          stack.pop_back();
          p = e + 1;
          continue;
        }
        // start tag
        p++;
        auto node = std::make_unique<XmlNode>();
        node->name = local(read_name());
        bool self_close = false;
        while (true) {
          skip_ws();
          if (p >= s->size()) throw ZbError("unterminated start tag");
          if ((*s)[p] == '/') { self_close = true; p++; continue; }
          if ((*s)[p] == '>') { p++; break; }
          std::string an = read_name();
          skip_ws();
          if (p >= s->size() || (*s)[p] != '=') throw ZbError("attribute without value");
          p++;
          skip_ws();
          char q = (*s)[p];
          if (q != '"' && q != '\'') throw ZbError("unquoted attribute");
          size_t e = s->find(q, p + 1);
          if (e == std::string::npos) throw ZbError("unterminated attribute");
          std::string v = decode(s->substr(p + 1, e - p - 1));
          p = e + 1;
          if (an.rfind("xmlns", 0) == 0) continue;
          node->attrs.emplace_back(local(an), v);
        }
        XmlNode* raw = node.get();
        raw->parent = stack.back();
        stack.back()->children.push_back(std::move(node));
        if (!self_close) stack.push_back(raw);
      } else {
        size_t e = s->find('<', p);
        if (e == std::string::npos) e = s->size();
        stack.back()->text += decode(s->substr(p, e - p));
        p = e;
      }
    }
    if (stack.size() != 1) throw ZbError("unclosed element");
    return root;
  }

 private:
  const std::string* s = nullptr;
  size_t p = 0;
  bool starts(const char* t) const { return s->compare(p, std::strlen(t), t) == 0; }
  void skip_to(const char* t) {
    size_t e = s->find(t, p);
    if (e == std::string::npos) throw ZbError("unterminated markup");
    p = e + std::strlen(t);
  }
  void skip_ws() {
    while (p < s->size() && ((*s)[p] == ' ' || (*s)[p] == '\t' || (*s)[p] == '\n' || (*s)[p] == '\r')) p++;
  }
  std::string read_name() {
    size_t b = p;
    while (p < s->size()) {
      char c = (*s)[p];
      if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '/' || c == '>' || c == '=') break;
      p++;
    }
    return s->substr(b, p - b);
  }
  static std::string local(const std::string& n) {
    size_t i = n.find(':');
    return i == std::string::npos ? n : n.substr(i + 1);
  }
  static void put_utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) o.push_back((char)cp);
    else if (cp < 0x800) { o.push_back((char)(0xc0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3f))); }
    else if (cp < 0x10000) {
      o.push_back((char)(0xe0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
      o.push_back((char)(0x80 | (cp & 0x3f)));
    } else {
      o.push_back((char)(0xf0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3f)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3f))); o.push_back((char)(0x80 | (cp & 0x3f)));
    }
  }
  static std::string decode(const std::string& in) {
    std::string o;
    for (size_t i = 0; i < in.size(); i++) {
      if (in[i] != '&') { o.push_back(in[i]); continue; }
      size_t e = in.find(';', i);
      if (e == std::string::npos) { o.push_back('&'); continue; }
      std::string ent = in.substr(i + 1, e - i - 1);
      if (ent == "lt") o.push_back('<');
      else if (ent == "gt") o.push_back('>');
      else if (ent == "amp") o.push_back('&');
      else if (ent == "quot") o.push_back('"');
      else if (ent == "apos") o.push_back('\'');
      else if (!ent.empty() && ent[0] == '#') {
        unsigned cp = ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X') ? (unsigned)std::stoul(ent.substr(2), nullptr, 16)
                                                                          : (unsigned)std::stoul(ent.substr(1));
        put_utf8(o, cp);
      } else { o += "&" + ent + ";"; }
      i = e;
    }
    return o;
  }
};

}  // namespace zbref
