// json_min.hpp — minimal JSON reader for scene files (RFC 8259 subset: objects,
// arrays, strings with the standard escapes, numbers, true/false/null).  Object
// members keep their file order (the scene loader assigns table indices in
// reference order, see scene_json.hpp).
#pragma once

#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace jsonmin {

struct Value {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  bool is_object() const { return kind == Object; }
  bool is_array() const { return kind == Array; }
  bool is_string() const { return kind == String; }
  bool is_number() const { return kind == Number; }
  const Value *find(const std::string &k) const {
    for (const auto &kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  bool has(const std::string &k) const { return find(k) != nullptr; }
  const Value &at(const std::string &k) const {
    const Value *v = find(k);
    if (!v) throw std::runtime_error("missing key '" + k + "'");
    return *v;
  }
  double number() const {
    if (kind == Number) return num;
    if (kind == Bool) return b ? 1 : 0;
    throw std::runtime_error("expected a number");
  }
};

class Parser {
public:
  explicit Parser(const std::string &s) : s_(s) {}
  Value parse() {
    Value v = value();
    ws();
    if (i_ != s_.size()) fail("trailing characters");
    return v;
  }

private:
  const std::string &s_;
  size_t i_ = 0;
  // Nesting bound: value() recurses per array/object level, so an adversarial
  // file ("[[[[...") would otherwise overflow the stack (found by make sanitize).
  static constexpr int kMaxDepth = 256;
  int depth_ = 0;
  struct Nest {
    Parser &p;
    explicit Nest(Parser &q) : p(q) {
      if (++p.depth_ > kMaxDepth) p.fail("nesting deeper than 256 levels");
    }
    ~Nest() { --p.depth_; }
  };

  [[noreturn]] void fail(const std::string &m) {
    throw std::runtime_error("JSON parse error at offset " + std::to_string(i_) + ": " + m);
  }
  void ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r'))
      ++i_;
  }
  bool lit(const char *w) {
    size_t n = std::char_traits<char>::length(w);
    if (s_.compare(i_, n, w) == 0) {
      i_ += n;
      return true;
    }
    return false;
  }
  Value value() {
    Nest guard(*this);
    ws();
    if (i_ >= s_.size()) fail("unexpected end");
    char c = s_[i_];
    Value v;
    if (c == '{') {
      v.kind = Value::Object;
      ++i_;
      ws();
      if (i_ < s_.size() && s_[i_] == '}') {
        ++i_;
        return v;
      }
      for (;;) {
        ws();
        if (i_ >= s_.size() || s_[i_] != '"') fail("expected key");
        std::string k = string();
        ws();
        if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
        ++i_;
        v.obj.emplace_back(k, value());
        ws();
        if (i_ < s_.size() && s_[i_] == ',') {
          ++i_;
          continue;
        }
        if (i_ < s_.size() && s_[i_] == '}') {
          ++i_;
          return v;
        }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      v.kind = Value::Array;
      ++i_;
      ws();
      if (i_ < s_.size() && s_[i_] == ']') {
        ++i_;
        return v;
      }
      for (;;) {
        v.arr.push_back(value());
        ws();
        if (i_ < s_.size() && s_[i_] == ',') {
          ++i_;
          continue;
        }
        if (i_ < s_.size() && s_[i_] == ']') {
          ++i_;
          return v;
        }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v.kind = Value::String;
      v.str = string();
      return v;
    }
    if (lit("true")) {
      v.kind = Value::Bool;
      v.b = true;
      return v;
    }
    if (lit("false")) {
      v.kind = Value::Bool;
      return v;
    }
    if (lit("null")) return v;
    const char *start = s_.c_str() + i_;
    char *end = nullptr;
    double d = std::strtod(start, &end);
    if (end == start) fail("bad value");
    i_ += size_t(end - start);
    v.kind = Value::Number;
    v.num = d;
    return v;
  }
  std::string string() {
    ++i_; // opening quote
    std::string out;
    while (i_ < s_.size() && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\') {
        if (i_ >= s_.size()) fail("bad escape");
        char e = s_[i_++];
        switch (e) {
        case 'n': out += '\n'; break;
        case 't': out += '\t'; break;
        case 'r': out += '\r'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'u': {
          if (i_ + 4 > s_.size()) fail("bad \\u escape");
          unsigned cp = std::stoul(s_.substr(i_, 4), nullptr, 16);
          i_ += 4;
          if (cp < 0x80) out += char(cp);
          else if (cp < 0x800) {
            out += char(0xC0 | (cp >> 6));
            out += char(0x80 | (cp & 63));
          } else {
            out += char(0xE0 | (cp >> 12));
            out += char(0x80 | ((cp >> 6) & 63));
            out += char(0x80 | (cp & 63));
          }
          break;
        }
        default: out += e;
        }
      } else {
        out += c;
      }
    }
    if (i_ >= s_.size()) fail("unterminated string");
    ++i_;
    return out;
  }
};

inline Value parse(const std::string &text) { return Parser(text).parse(); }

} // namespace jsonmin
