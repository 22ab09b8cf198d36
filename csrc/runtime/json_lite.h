// Minimal JSON DOM parser for request bodies (RFC 8259 subset sufficient for API payloads:
// objects, arrays, strings with escapes incl. \uXXXX, numbers, true/false/null).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace rtj {

struct Value {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0.0;
  bool is_int = false;
  std::string str;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  const Value* get(const char* key) const {
    if (kind != Obj) return nullptr;
    for (const auto& kv : obj)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
  // Python truthiness
  bool truthy() const {
    switch (kind) {
      case Null: return false;
      case Bool: return b;
      case Num: return num != 0.0;
      case Str: return !str.empty();
      case Arr: return !arr.empty();
      case Obj: return !obj.empty();
    }
    return false;
  }
};

class Parser {
 public:
  Parser(const char* s, size_t n) : p_(s), e_(s + n) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != e_) fail("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  int depth_ = 0;

  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("invalid JSON: ") + m); }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  bool lit(const char* s) {
    size_t n = std::strlen(s);
    if ((size_t)(e_ - p_) >= n && std::memcmp(p_, s, n) == 0) {
      p_ += n;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& o, uint32_t c) {
    if (c < 0x80) o += (char)c;
    else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 0x3F)); }
    else if (c < 0x10000) {
      o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F));
    } else {
      o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3F));
      o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F));
    }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) fail("short \\u escape");
    uint32_t c = 0;
    for (int i = 0; i < 4; ++i) {
      char h = *p_++;
      c <<= 4;
      if (h >= '0' && h <= '9') c |= h - '0';
      else if (h >= 'a' && h <= 'f') c |= h - 'a' + 10;
      else if (h >= 'A' && h <= 'F') c |= h - 'A' + 10;
      else fail("bad hex");
    }
    return c;
  }
  std::string string() {
    if (p_ >= e_ || *p_ != '"') fail("expected string");
    ++p_;
    std::string o;
    while (true) {
      if (p_ >= e_) fail("unterminated string");
      char c = *p_++;
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control char in string");
      if (c != '\\') { o += c; continue; }
      if (p_ >= e_) fail("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return o;
  }
  Value value() {
    ws();
    if (p_ >= e_) fail("unexpected end");
    Value v;
    char c = *p_;
    if (c == '{') {
      if (++depth_ > 64) fail("too deep");
      ++p_;
      v.kind = Value::Obj;
      ws();
      if (p_ < e_ && *p_ == '}') { ++p_; --depth_; return v; }
      while (true) {
        ws();
        std::string k = string();
        ws();
        if (p_ >= e_ || *p_ != ':') fail("expected ':'");
        ++p_;
        Value item = value();
        bool replaced = false;   // duplicate keys: last one wins (Python json)
        for (auto& kv : v.obj)
          if (kv.first == k) { kv.second = std::move(item); replaced = true; break; }
        if (!replaced) v.obj.emplace_back(std::move(k), std::move(item));
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; break; }
        fail("expected ',' or '}'");
      }
      --depth_;
    } else if (c == '[') {
      if (++depth_ > 64) fail("too deep");
      ++p_;
      v.kind = Value::Arr;
      ws();
      if (p_ < e_ && *p_ == ']') { ++p_; --depth_; return v; }
      while (true) {
        v.arr.push_back(value());
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; break; }
        fail("expected ',' or ']'");
      }
      --depth_;
    } else if (c == '"') {
      v.kind = Value::Str;
      v.str = string();
    } else if (lit("true")) {
      v.kind = Value::Bool;
      v.b = true;
    } else if (lit("false")) {
      v.kind = Value::Bool;
    } else if (lit("null")) {
      v.kind = Value::Null;
    } else if (lit("NaN")) {                       // Python json accepts these
      v.kind = Value::Num; v.num = NAN;
    } else if (lit("Infinity")) {
      v.kind = Value::Num; v.num = INFINITY;
    } else if (lit("-Infinity")) {
      v.kind = Value::Num; v.num = -INFINITY;
    } else {
      const char* st = p_;
      if (p_ < e_ && *p_ == '-') ++p_;
      bool is_int = true;
      while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                         *p_ == '+' || *p_ == '-')) {
        if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') is_int = false;
        ++p_;
      }
      if (p_ == st) fail("unexpected character");
      std::string tok(st, p_);
      char* endp = nullptr;
      v.num = std::strtod(tok.c_str(), &endp);
      if (endp != tok.c_str() + tok.size()) fail("bad number");
      v.kind = Value::Num;
      v.is_int = is_int;
    }
    return v;
  }
};

}  // namespace rtj
