// SeldonMessage data model + JSON / protobuf wire codecs.
//
// Wire-compatible with proto/prediction.proto (reference
// proto/prediction.proto:14-128).  The engine keeps one C++ struct per
// message; numeric payloads are exposed as a dense (shape, fp64 values) view so
// GPU nodes can stage them straight into pinned/HBM buffers without touching a
// DOM (reference decode hot path: python/seldon_core/utils.py:147-181,
// engine/.../PredictorUtils.java:34-195).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "json.h"

namespace sca {

struct CodecError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

enum class MetricType : int32_t { COUNTER = 0, GAUGE = 1, TIMER = 2 };
const char* metric_type_name(MetricType t);

using StrMap = std::vector<std::pair<std::string, std::string>>;

struct Metric {
  std::string key;
  MetricType type = MetricType::COUNTER;
  float value = 0.f;
  StrMap tags;
};

struct Meta {
  std::string puid;
  Json::Object tags;  // map<string, google.protobuf.Value>, insertion ordered
  std::vector<std::pair<std::string, int32_t>> routing;
  StrMap request_path;
  std::vector<Metric> metrics;

  void put_tag(const std::string& k, Json v);
  void put_routing(const std::string& k, int32_t v);
  void put_request_path(const std::string& k, const std::string& v);
  const Json* tag(std::string_view k) const;
  bool routing_of(std::string_view k, int32_t& out) const;
};

struct Status {
  int32_t code = 0;
  std::string info;
  std::string reason;
  int32_t status = 0;  // 0 SUCCESS, 1 FAILURE
};

// tensorflow.TensorProto subset (reference tensorflow/core/framework/tensor.proto)
enum TfDType : int32_t {
  DT_INVALID = 0, DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4,
  DT_INT16 = 5, DT_INT8 = 6, DT_STRING = 7, DT_COMPLEX64 = 8, DT_INT64 = 9,
  DT_BOOL = 10, DT_BFLOAT16 = 14, DT_UINT16 = 17, DT_COMPLEX128 = 18,
  DT_HALF = 19, DT_UINT32 = 22, DT_UINT64 = 23
};
const char* tf_dtype_name(int32_t dt);
int32_t tf_dtype_from_name(std::string_view s);

struct TfTensor {
  int32_t dtype = 0;
  std::vector<int64_t> dims;
  bool unknown_rank = false;
  int32_t version_number = 0;
  std::string content;  // tensor_content
  std::vector<float> float_val;
  std::vector<double> double_val;
  std::vector<int32_t> int_val;
  std::vector<std::string> string_val;
  std::vector<float> scomplex_val;
  std::vector<int64_t> int64_val;
  std::vector<uint8_t> bool_val;
  std::vector<double> dcomplex_val;
  std::vector<int32_t> half_val;
  std::vector<uint32_t> uint32_val;
  std::vector<uint64_t> uint64_val;

  // Numeric view (broadcasts a single *_val element as TF does).
  bool to_dense(std::vector<int64_t>& shape, std::vector<double>& v, std::string* err) const;
  static TfTensor from_dense(const std::vector<int64_t>& shape, const double* v, size_t n);
};

enum class DataKind : uint8_t { None, Tensor, NdArray, TfTensor };

struct DefaultData {
  std::vector<std::string> names;
  DataKind kind = DataKind::None;
  // Tensor payload, or a numeric ndarray held densely (nd_dense == true).
  std::vector<int64_t> shape;
  std::vector<double> values;
  bool nd_dense = false;
  Json ndarray;  // ListValue (generic ndarray, nd_dense == false)
  TfTensor tftensor;

  // Dense numeric view of any kind. Returns false (with err) for
  // non-rectangular or non-numeric payloads.
  bool dense(std::vector<int64_t>& shp, std::vector<double>& vals, std::string* err) const;
  // Replace the payload with dense values, keeping the current kind
  // (tensor / ndarray / tftensor).  Mirrors PredictorUtils.updateData.
  void set_dense(DataKind k, std::vector<int64_t> shp, std::vector<double> vals);
  int64_t rows() const;
};

enum class Payload : uint8_t { None, Data, BinData, StrData, JsonData };

struct SeldonMessage {
  bool has_status = false;
  Status status;
  bool has_meta = false;
  Meta meta;
  Payload payload = Payload::None;
  DefaultData data;
  std::string bin_data;
  std::string str_data;
  Json json_data;
};
using MsgPtr = std::shared_ptr<SeldonMessage>;

struct Feedback {
  bool has_request = false, has_response = false, has_truth = false;
  SeldonMessage request, response, truth;
  float reward = 0.f;
};

// ------------------------------------------------------------------ JSON codec
void message_from_json(const Json& j, SeldonMessage& m);
// Fast path for the dominant REST request shape, {"data": {["names": [..],]
// "ndarray": [[numbers], ...]}[, "meta": {}]} in any key order: parses
// straight into a dense ndarray (no JSON tree) with the same numbers and the
// same message as message_from_json(parse_json(text)).  Returns false, m
// untouched, for anything else (other fields, escapes, non-numbers, ragged
// or 1-D arrays, duplicate keys): the caller then takes the general parser.
bool fast_dense_message(std::string_view text, SeldonMessage& m);
void message_to_json(const SeldonMessage& m, std::string& out);
void feedback_from_json(const Json& j, Feedback& f);
void feedback_to_json(const Feedback& f, std::string& out);
void message_list_from_json(const Json& j, std::vector<SeldonMessage>& out);
void message_list_to_json(const std::vector<const SeldonMessage*>& msgs, std::string& out);
void status_to_json(const Status& s, std::string& out);
Json message_to_json_value(const SeldonMessage& m);  // convenience (DOM)

// -------------------------------------------------------------- protobuf codec
bool message_from_pb(std::string_view buf, SeldonMessage& m);
void message_to_pb(const SeldonMessage& m, std::string& out);
bool feedback_from_pb(std::string_view buf, Feedback& f);
void feedback_to_pb(const Feedback& f, std::string& out);
bool message_list_from_pb(std::string_view buf, std::vector<SeldonMessage>& out);
void message_list_to_pb(const std::vector<const SeldonMessage*>& msgs, std::string& out);

}  // namespace sca
