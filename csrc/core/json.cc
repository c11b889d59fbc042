#include "json.h"

#include <charconv>
#include <cmath>
#include <cstring>

namespace sca {

// ---------------------------------------------------------------- object ops
const Json* Json::find(std::string_view key) const {
  if (type_ != Type::Object) return nullptr;
  for (const auto& m : o_)
    if (m.first == key) return &m.second;
  return nullptr;
}

Json* Json::find(std::string_view key) {
  if (type_ != Type::Object) return nullptr;
  for (auto& m : o_)
    if (m.first == key) return &m.second;
  return nullptr;
}

Json& Json::operator[](std::string_view key) {
  if (type_ == Type::Null) type_ = Type::Object;
  if (Json* j = find(key)) return *j;
  o_.emplace_back(std::string(key), Json());
  return o_.back().second;
}

void Json::set(std::string_view key, Json v) { (*this)[key] = std::move(v); }

bool Json::erase(std::string_view key) {
  for (auto it = o_.begin(); it != o_.end(); ++it)
    if (it->first == key) { o_.erase(it); return true; }
  return false;
}

bool Json::operator==(const Json& o) const {
  if (type_ != o.type_) return false;
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::Number: return n_ == o.n_;
    case Type::String: return s_ == o.s_;
    case Type::Array: return a_ == o.a_;
    case Type::Object: {
      if (o_.size() != o.o_.size()) return false;
      for (const auto& m : o_) {
        const Json* other = o.find(m.first);
        if (!other || !(*other == m.second)) return false;
      }
      return true;
    }
  }
  return false;
}

std::string Json::dump() const {
  std::string out;
  write_json(*this, out);
  return out;
}

// ------------------------------------------------------------------- numbers
static const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

bool parse_double(const char* b, const char* e, double& out) {
  // Clinger's fast path: exact when the decimal mantissa fits in 53 bits and
  // |exp10| <= 22.  Covers nearly every feature value on the wire.
  const char* p = b;
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) { neg = (*p == '-'); ++p; }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool any = false;
  while (p < e && *p >= '0' && *p <= '9') {
    any = true;
    if (digits < 19) { mant = mant * 10 + uint64_t(*p - '0'); if (mant) ++digits; }
    else ++exp10;
    ++p;
  }
  if (p < e && *p == '.') {
    ++p;
    while (p < e && *p >= '0' && *p <= '9') {
      any = true;
      if (digits < 19) { mant = mant * 10 + uint64_t(*p - '0'); if (mant) ++digits; --exp10; }
      ++p;
    }
  }
  if (!any) return false;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '-' || *p == '+')) { eneg = (*p == '-'); ++p; }
    int ev = 0;
    bool edig = false;
    while (p < e && *p >= '0' && *p <= '9') { edig = true; if (ev < 100000) ev = ev * 10 + (*p - '0'); ++p; }
    if (!edig) return false;
    exp10 += eneg ? -ev : ev;
  }
  if (p != e) return false;
  if (mant < (uint64_t(1) << 53) && exp10 >= -22 && exp10 <= 22) {
    double d = double(mant);
    d = exp10 >= 0 ? d * kPow10[exp10] : d / kPow10[-exp10];
    out = neg ? -d : d;
    return true;
  }
  const char* fb = (*b == '+') ? b + 1 : b;
  auto r = std::from_chars(fb, e, out);
  if (r.ec == std::errc::result_out_of_range) {
    out = neg ? -HUGE_VAL : HUGE_VAL;
    if (exp10 < 0) out = neg ? -0.0 : 0.0;
    return true;
  }
  return r.ec == std::errc() && r.ptr == e;
}

void append_number(std::string& out, double v) {
  if (std::isnan(v)) { out += "\"NaN\""; return; }
  if (std::isinf(v)) { out += v > 0 ? "\"Infinity\"" : "\"-Infinity\""; return; }
  char buf[40];
  if (v == std::floor(v) && std::fabs(v) < 1e15) {
    auto r = std::to_chars(buf, buf + sizeof buf, int64_t(v));
    out.append(buf, r.ptr);
    out += ".0";
    return;
  }
  auto r = std::to_chars(buf, buf + sizeof buf, v);
  out.append(buf, r.ptr);
}

void append_float(std::string& out, float v) {
  if (std::isnan(v)) { out += "\"NaN\""; return; }
  if (std::isinf(v)) { out += v > 0 ? "\"Infinity\"" : "\"-Infinity\""; return; }
  char buf[40];
  if (v == std::floor(v) && std::fabs(v) < 1e7f) {
    auto r = std::to_chars(buf, buf + sizeof buf, int64_t(v));
    out.append(buf, r.ptr);
    out += ".0";
    return;
  }
  auto r = std::to_chars(buf, buf + sizeof buf, v);
  out.append(buf, r.ptr);
}

void append_quoted(std::string& out, std::string_view s) {
  static const char* hex = "0123456789abcdef";
  out.push_back('"');
  size_t run = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    unsigned char c = (unsigned char)s[i];
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(s.data() + run, i - run);
    run = i + 1;
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        out += "\\u00";
        out.push_back(hex[c >> 4]);
        out.push_back(hex[c & 15]);
    }
  }
  out.append(s.data() + run, s.size() - run);
  out.push_back('"');
}

// -------------------------------------------------------------------- writer
void write_json(const Json& j, std::string& out) {
  switch (j.type()) {
    case Json::Type::Null: out += "null"; break;
    case Json::Type::Bool: out += j.as_bool() ? "true" : "false"; break;
    case Json::Type::Number: append_number(out, j.as_number()); break;
    case Json::Type::String: append_quoted(out, j.as_string()); break;
    case Json::Type::Array: {
      out.push_back('[');
      bool first = true;
      for (const auto& v : j.items()) {
        if (!first) out.push_back(',');
        first = false;
        write_json(v, out);
      }
      out.push_back(']');
      break;
    }
    case Json::Type::Object: {
      out.push_back('{');
      bool first = true;
      for (const auto& m : j.members()) {
        if (!first) out.push_back(',');
        first = false;
        append_quoted(out, m.first);
        out.push_back(':');
        write_json(m.second, out);
      }
      out.push_back('}');
      break;
    }
  }
}

// -------------------------------------------------------------------- parser
namespace {

struct Parser {
  const char* p;
  const char* e;
  int depth = 0;

  [[noreturn]] void fail(const char* what) {
    throw JsonError(std::string("invalid JSON: ") + what);
  }
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) s.push_back(char(cp));
    else if (cp < 0x800) { s.push_back(char(0xC0 | (cp >> 6))); s.push_back(char(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
      s.push_back(char(0xE0 | (cp >> 12)));
      s.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      s.push_back(char(0x80 | (cp & 0x3F)));
    } else {
      s.push_back(char(0xF0 | (cp >> 18)));
      s.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
      s.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      s.push_back(char(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t hex4() {
    if (e - p < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      int h = hexv(p[i]);
      if (h < 0) fail("bad \\u escape");
      v = (v << 4) | uint32_t(h);
    }
    p += 4;
    return v;
  }
  std::string str() {
    // assumes *p == '"'
    ++p;
    std::string s;
    const char* run = p;
    while (true) {
      if (p >= e) fail("unterminated string");
      char c = *p;
      if (c == '"') { s.append(run, p); ++p; return s; }
      if (c == '\\') {
        s.append(run, p);
        ++p;
        if (p >= e) fail("bad escape");
        char x = *p++;
        switch (x) {
          case '"': s.push_back('"'); break;
          case '\\': s.push_back('\\'); break;
          case '/': s.push_back('/'); break;
          case 'b': s.push_back('\b'); break;
          case 'f': s.push_back('\f'); break;
          case 'n': s.push_back('\n'); break;
          case 'r': s.push_back('\r'); break;
          case 't': s.push_back('\t'); break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(s, cp);
            break;
          }
          default: fail("bad escape");
        }
        run = p;
        continue;
      }
      if ((unsigned char)c < 0x20) fail("control character in string");
      ++p;
    }
  }
  Json value() {
    ws();
    if (p >= e) fail("unexpected end");
    char c = *p;
    if (c == '{') {
      if (++depth > 512) fail("nesting too deep");
      ++p;
      Json j = Json::object();
      ws();
      if (p < e && *p == '}') { ++p; --depth; return j; }
      while (true) {
        ws();
        if (p >= e || *p != '"') fail("expected key");
        std::string k = str();
        ws();
        if (p >= e || *p != ':') fail("expected ':'");
        ++p;
        j.members().emplace_back(std::move(k), value());
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; break; }
        fail("expected ',' or '}'");
      }
      --depth;
      return j;
    }
    if (c == '[') {
      if (++depth > 512) fail("nesting too deep");
      ++p;
      Json j = Json::array();
      ws();
      if (p < e && *p == ']') { ++p; --depth; return j; }
      while (true) {
        j.items().push_back(value());
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; break; }
        fail("expected ',' or ']'");
      }
      --depth;
      return j;
    }
    if (c == '"') return Json(str());
    if (c == 't') { if (e - p >= 4 && !memcmp(p, "true", 4)) { p += 4; return Json(true); } fail("bad literal"); }
    if (c == 'f') { if (e - p >= 5 && !memcmp(p, "false", 5)) { p += 5; return Json(false); } fail("bad literal"); }
    if (c == 'n') { if (e - p >= 4 && !memcmp(p, "null", 4)) { p += 4; return Json(); } fail("bad literal"); }
    if (c == 'N' && e - p >= 3 && !memcmp(p, "NaN", 3)) { p += 3; return Json(std::nan("")); }
    if (c == 'I' && e - p >= 8 && !memcmp(p, "Infinity", 8)) { p += 8; return Json(HUGE_VAL); }
    if (c == '-' && e - p >= 9 && !memcmp(p, "-Infinity", 9)) { p += 9; return Json(-HUGE_VAL); }
    const char* b = p;
    if (p < e && (*p == '-')) ++p;
    while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) ++p;
    if (b == p) fail("unexpected character");
    double d;
    if (!parse_double(b, p, d)) fail("bad number");
    return Json(d);
  }
};

}  // namespace

Json parse_json(std::string_view text) {
  Parser ps{text.data(), text.data() + text.size()};
  Json j = ps.value();
  ps.ws();
  if (ps.p != ps.e) ps.fail("trailing characters");
  return j;
}

// -------------------------------------------------------------------- base64
static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(std::string_view raw) {
  std::string out;
  out.reserve((raw.size() + 2) / 3 * 4);
  size_t i = 0;
  const unsigned char* s = (const unsigned char*)raw.data();
  for (; i + 2 < raw.size(); i += 3) {
    uint32_t v = (s[i] << 16) | (s[i + 1] << 8) | s[i + 2];
    out.push_back(kB64[v >> 18]);
    out.push_back(kB64[(v >> 12) & 63]);
    out.push_back(kB64[(v >> 6) & 63]);
    out.push_back(kB64[v & 63]);
  }
  if (i < raw.size()) {
    uint32_t v = s[i] << 16;
    if (i + 1 < raw.size()) v |= s[i + 1] << 8;
    out.push_back(kB64[v >> 18]);
    out.push_back(kB64[(v >> 12) & 63]);
    out.push_back(i + 1 < raw.size() ? kB64[(v >> 6) & 63] : '=');
    out.push_back('=');
  }
  return out;
}

bool base64_decode(std::string_view b64, std::string& out) {
  static int8_t table[256];
  static bool init = [] {
    memset(table, -1, sizeof table);
    for (int i = 0; i < 64; ++i) table[(unsigned char)kB64[i]] = int8_t(i);
    table[(unsigned char)'-'] = 62;  // url-safe alphabet accepted too
    table[(unsigned char)'_'] = 63;
    return true;
  }();
  (void)init;
  out.clear();
  out.reserve(b64.size() * 3 / 4);
  uint32_t acc = 0;
  int bits = 0;
  for (char c : b64) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ') continue;
    int v = table[(unsigned char)c];
    if (v < 0) return false;
    acc = (acc << 6) | uint32_t(v);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back(char((acc >> bits) & 0xFF));
    }
  }
  return true;
}

}  // namespace sca
