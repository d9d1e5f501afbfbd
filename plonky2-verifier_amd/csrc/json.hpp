// json.hpp — small DOM JSON reader for the Types.hs wire format (reference
// src/Types.hs:70-279).  Numbers keep their text so arbitrary-size integers reduce mod p
// exactly like aeson Integer + mkGoldilocks (Goldilocks.hs:98-102).
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace p2v {

struct ParseError : std::runtime_error { using std::runtime_error::runtime_error; };
struct ShapeError : std::runtime_error { using std::runtime_error::runtime_error; };
struct CircuitError : std::runtime_error { using std::runtime_error::runtime_error; };

// characters of a number token (the reader is permissive; typed accessors validate)
inline bool is_num_char(char c) { return (c >= '0' && c <= '9') || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-'; }

struct JVal {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  std::string text;                    // number text / string value
  std::vector<JVal> items;             // array items / object values
  std::vector<std::string> keys;       // object keys
  int32_t ord = -1;                    // number: ordinal in document order

  const JVal* get(const char* k) const {
    if (kind != Obj) return nullptr;
    for (size_t i = 0; i < keys.size(); i++) if (keys[i] == k) return &items[i];
    return nullptr;
  }
  const JVal& at(const char* k) const {
    const JVal* v = get(k);
    if (!v) throw ParseError(std::string("missing key `") + k + "`");
    return *v;
  }
  const std::vector<JVal>& arr() const {
    if (kind != Arr) throw ParseError("expected array");
    return items;
  }
};

class JParser {
 public:
  JParser(const char* s, size_t n, std::vector<std::pair<size_t, size_t>>* spans = nullptr) : s_(s), n_(n), spans_(spans) {}
  JVal parse() {
    JVal v; value(v); ws();
    if (i_ != n_) throw ParseError("trailing characters after JSON value");
    return v;
  }
 private:
  const char* s_; size_t n_, i_ = 0;
  std::vector<std::pair<size_t, size_t>>* spans_;   // number token [start, end) by ordinal
  int32_t nnum_ = 0;
  void ws() { while (i_ < n_ && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) i_++; }
  [[noreturn]] void bad(const char* m) { throw ParseError(std::string("JSON syntax: ") + m + " at offset " + std::to_string(i_)); }
  void str(std::string& out) {
    i_++;
    while (i_ < n_ && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\') {
        if (i_ >= n_) bad("bad escape");
        char e = s_[i_++];
        switch (e) {
          case 'n': c = '\n'; break; case 't': c = '\t'; break; case 'r': c = '\r'; break;
          case 'b': c = '\b'; break; case 'f': c = '\f'; break;
          case 'u': { if (i_ + 4 > n_) bad("bad \\u"); unsigned v = (unsigned)std::stoul(std::string(s_ + i_, 4), nullptr, 16); i_ += 4; c = (char)(v < 128 ? v : '?'); break; }
          default: c = e;
        }
      }
      out.push_back(c);
    }
    if (i_ >= n_) bad("unterminated string");
    i_++;
  }
  void value(JVal& v) {
    ws();
    if (i_ >= n_) bad("unexpected end");
    char c = s_[i_];
    if (c == '{') {
      v.kind = JVal::Obj; i_++; ws();
      if (i_ < n_ && s_[i_] == '}') { i_++; return; }
      for (;;) {
        ws(); if (i_ >= n_ || s_[i_] != '"') bad("expected key");
        v.keys.emplace_back(); str(v.keys.back());
        ws(); if (i_ >= n_ || s_[i_] != ':') bad("expected ':'"); i_++;
        v.items.emplace_back(); value(v.items.back());
        ws(); if (i_ < n_ && s_[i_] == ',') { i_++; continue; }
        if (i_ < n_ && s_[i_] == '}') { i_++; return; }
        bad("expected ',' or '}'");
      }
    }
    if (c == '[') {
      v.kind = JVal::Arr; i_++; ws();
      if (i_ < n_ && s_[i_] == ']') { i_++; return; }
      for (;;) {
        v.items.emplace_back(); value(v.items.back());
        ws(); if (i_ < n_ && s_[i_] == ',') { i_++; continue; }
        if (i_ < n_ && s_[i_] == ']') { i_++; return; }
        bad("expected ',' or ']'");
      }
    }
    if (c == '"') { v.kind = JVal::Str; str(v.text); return; }
    if (!strncmp(s_ + i_, "true", 4) && i_ + 4 <= n_) { v.kind = JVal::Bool; v.b = true; i_ += 4; return; }
    if (!strncmp(s_ + i_, "false", 5) && i_ + 5 <= n_) { v.kind = JVal::Bool; i_ += 5; return; }
    if (!strncmp(s_ + i_, "null", 4) && i_ + 4 <= n_) { v.kind = JVal::Null; i_ += 4; return; }
    if (c == '-' || (c >= '0' && c <= '9')) {
      size_t st = i_++;
      while (i_ < n_ && is_num_char(s_[i_])) i_++;
      v.kind = JVal::Num; v.text.assign(s_ + st, i_ - st); v.ord = nnum_++;
      if (spans_) spans_->emplace_back(st, i_);
      return;
    }
    bad("unexpected character");
  }
};

inline JVal parse_json(const char* s, size_t n) { return JParser(s, n).parse(); }

// ---- typed accessors ---------------------------------------------------------------
static constexpr uint64_t GL_P = 0xFFFFFFFF00000001ULL;

// aeson Integer -> mod p (negative numbers reduce to the non-negative residue).
// Number token text [s, s+n) -> false if it is not an integer.
inline bool field_of_text(const char* s, size_t n, uint64_t& out) {
  size_t i = 0; bool neg = false;
  if (n && s[0] == '-') { neg = true; i = 1; }
  if (i >= n) return false;
  uint64_t acc = 0;
  // up to 19 digits accumulate exactly in 64 bits; longer integers reduce as they go
  for (; i < n; i++) {
    const unsigned d = (unsigned)(s[i] - '0');
    if (d > 9) return false;
    if (acc < 1000000000000000000ULL) acc = acc * 10 + d;
    else acc = (uint64_t)(((unsigned __int128)acc * 10 + d) % GL_P);
  }
  if (acc >= GL_P) acc -= GL_P;
  out = (neg && acc) ? GL_P - acc : acc;
  return true;
}
inline uint64_t j_field(const JVal& v) {
  if (v.kind != JVal::Num) throw ParseError("expected an integer field element");
  uint64_t r;
  if (v.text.empty() || (v.text[0] == '-' && v.text.size() == 1)) throw ParseError("bad number");
  if (!field_of_text(v.text.data(), v.text.size(), r)) throw ParseError("non-integral number where a field element is expected");
  return r;
}
inline int64_t j_int(const JVal& v) {
  if (v.kind != JVal::Num) throw ParseError("expected an integer");
  for (size_t i = 0; i < v.text.size(); i++) {
    char c = v.text[i];
    if (!((c >= '0' && c <= '9') || (i == 0 && c == '-'))) throw ParseError("non-integral number where Int is expected");
  }
  return std::stoll(v.text);
}
// an Int field this build stores as int: values outside int32 are rejected, never truncated
inline int j_i32(const JVal& v) {
  if (v.kind == JVal::Num && v.text.size() > 11) throw ParseError("Int field out of range");
  const int64_t x = j_int(v);
  if (x < INT32_MIN || x > INT32_MAX) throw ParseError("Int field out of range");
  return (int)x;
}
inline uint64_t j_word64_mod_p(const JVal& v) {   // Word64 then toF (Types.hs:30-35)
  if (v.kind != JVal::Num || v.text.empty() || v.text[0] == '-') throw ParseError("expected Word64");
  unsigned __int128 acc = 0;
  for (char c : v.text) {
    if (c < '0' || c > '9') throw ParseError("non-integral Word64");
    acc = acc * 10 + (unsigned)(c - '0');
    if (acc >> 64) throw ParseError("Word64 out of range");
  }
  return (uint64_t)(acc % GL_P);
}
inline bool j_bool(const JVal& v) { if (v.kind != JVal::Bool) throw ParseError("expected bool"); return v.b; }

}  // namespace p2v
