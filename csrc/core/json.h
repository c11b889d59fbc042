// Minimal, allocation-conscious JSON DOM used by the engine's wire codecs.
//
// The reference parses every hop with protobuf-java's JsonFormat
// (engine/src/main/java/io/seldon/engine/pb/ProtoBufUtils.java:42-75) and the
// Python wrapper with json_format (python/seldon_core/utils.py:17-117).  Here
// a single C++ DOM is shared by the REST front end, the message codec and the
// graph-spec loader so a request is parsed exactly once per process.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace sca {

struct JsonError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum class Type : uint8_t { Null, Bool, Number, String, Array, Object };
  using Array = std::vector<Json>;
  using Member = std::pair<std::string, Json>;
  using Object = std::vector<Member>;

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(double d) : type_(Type::Number), n_(d) {}
  Json(int v) : type_(Type::Number), n_(v) {}
  Json(int64_t v) : type_(Type::Number), n_(double(v)) {}
  Json(const char* s) : type_(Type::String), s_(s) {}
  Json(std::string s) : type_(Type::String), s_(std::move(s)) {}
  Json(std::string_view s) : type_(Type::String), s_(s) {}

  static Json array() { Json j; j.type_ = Type::Array; return j; }
  static Json object() { Json j; j.type_ = Type::Object; return j; }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Number; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const { return b_; }
  double as_number() const { return n_; }
  const std::string& as_string() const { return s_; }
  std::string& as_string() { return s_; }
  const Array& items() const { return a_; }
  Array& items() { return a_; }
  const Object& members() const { return o_; }
  Object& members() { return o_; }

  // Object helpers (linear scan: objects on this path are tiny).
  const Json* find(std::string_view key) const;
  Json* find(std::string_view key);
  Json& operator[](std::string_view key);  // insert-or-get (object only)
  void set(std::string_view key, Json v);   // replace-or-append
  bool erase(std::string_view key);
  void push_back(Json v) { a_.push_back(std::move(v)); }
  size_t size() const { return type_ == Type::Array ? a_.size() : o_.size(); }

  std::string dump() const;
  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  Type type_ = Type::Null;
  bool b_ = false;
  double n_ = 0.0;
  std::string s_;
  Array a_;
  Object o_;
};

Json parse_json(std::string_view text);
void write_json(const Json& j, std::string& out);

// Formatting primitives shared with the streaming encoders.
void append_number(std::string& out, double v);
void append_float(std::string& out, float v);
void append_quoted(std::string& out, std::string_view s);

std::string base64_encode(std::string_view raw);
bool base64_decode(std::string_view b64, std::string& out);

// Fast decimal parse (Clinger fast path + from_chars fallback).
bool parse_double(const char* b, const char* e, double& out);

}  // namespace sca
