// JSON codec for SeldonMessage / Feedback / SeldonMessageList.
//
// Parsing follows proto3 JSON mapping (accepts json_name and original field
// names, enum names or numbers, int64 as string or number, null == unset);
// printing follows the reference engine's printer configuration
// (`includingDefaultValueFields().preservingProtoFieldNames()`,
// engine/.../pb/ProtoBufUtils.java:42-60): Meta/Status/Metric/DefaultData are
// printed with their default-valued fields.
#include "message.h"

#include <cmath>
#include <cstring>

namespace sca {

const char* metric_type_name(MetricType t) {
  switch (t) {
    case MetricType::COUNTER: return "COUNTER";
    case MetricType::GAUGE: return "GAUGE";
    case MetricType::TIMER: return "TIMER";
  }
  return "COUNTER";
}

namespace {
struct DTypeName { int32_t v; const char* n; };
const DTypeName kDTypes[] = {
    {0, "DT_INVALID"}, {1, "DT_FLOAT"}, {2, "DT_DOUBLE"}, {3, "DT_INT32"},
    {4, "DT_UINT8"}, {5, "DT_INT16"}, {6, "DT_INT8"}, {7, "DT_STRING"},
    {8, "DT_COMPLEX64"}, {9, "DT_INT64"}, {10, "DT_BOOL"}, {11, "DT_QINT8"},
    {12, "DT_QUINT8"}, {13, "DT_QINT32"}, {14, "DT_BFLOAT16"}, {15, "DT_QINT16"},
    {16, "DT_QUINT16"}, {17, "DT_UINT16"}, {18, "DT_COMPLEX128"}, {19, "DT_HALF"},
    {20, "DT_RESOURCE"}, {21, "DT_VARIANT"}, {22, "DT_UINT32"}, {23, "DT_UINT64"}};
}  // namespace

const char* tf_dtype_name(int32_t dt) {
  for (const auto& d : kDTypes)
    if (d.v == dt) return d.n;
  return "DT_INVALID";
}

int32_t tf_dtype_from_name(std::string_view s) {
  for (const auto& d : kDTypes)
    if (s == d.n) return d.v;
  return -1;
}

// ---------------------------------------------------------------------- Meta
void Meta::put_tag(const std::string& k, Json v) {
  for (auto& m : tags)
    if (m.first == k) { m.second = std::move(v); return; }
  tags.emplace_back(k, std::move(v));
}
void Meta::put_routing(const std::string& k, int32_t v) {
  for (auto& m : routing)
    if (m.first == k) { m.second = v; return; }
  routing.emplace_back(k, v);
}
void Meta::put_request_path(const std::string& k, const std::string& v) {
  for (auto& m : request_path)
    if (m.first == k) { m.second = v; return; }
  request_path.emplace_back(k, v);
}
const Json* Meta::tag(std::string_view k) const {
  for (const auto& m : tags)
    if (m.first == k) return &m.second;
  return nullptr;
}
bool Meta::routing_of(std::string_view k, int32_t& out) const {
  for (const auto& m : routing)
    if (m.first == k) { out = m.second; return true; }
  return false;
}

// ------------------------------------------------------------- dense helpers
namespace {

bool json_shape(const Json& j, std::vector<int64_t>& shape) {
  const Json* cur = &j;
  while (cur->is_array()) {
    shape.push_back(int64_t(cur->items().size()));
    if (cur->items().empty()) break;
    cur = &cur->items()[0];
  }
  return true;
}

bool json_fill(const Json& j, const std::vector<int64_t>& shape, size_t d,
               std::vector<double>& out, std::string* err) {
  if (d == shape.size()) {
    if (!j.is_number()) {
      if (err) *err = "ndarray contains non-numeric values";
      return false;
    }
    out.push_back(j.as_number());
    return true;
  }
  if (!j.is_array() || int64_t(j.items().size()) != shape[d]) {
    if (err) *err = "ndarray is not rectangular";
    return false;
  }
  for (const auto& x : j.items())
    if (!json_fill(x, shape, d + 1, out, err)) return false;
  return true;
}

void write_dense_nd(std::string& out, const std::vector<int64_t>& shape,
                    const double* v, size_t d, size_t& off) {
  if (shape.empty()) {  // scalar payload: render as a single number
    append_number(out, v[off++]);
    return;
  }
  out.push_back('[');
  const int64_t n = shape[d];
  for (int64_t i = 0; i < n; ++i) {
    if (i) out.push_back(',');
    if (d + 1 == shape.size()) append_number(out, v[off++]);
    else write_dense_nd(out, shape, v, d + 1, off);
  }
  out.push_back(']');
}

Json dense_to_json(const std::vector<int64_t>& shape, const double* v, size_t d, size_t& off) {
  Json a = Json::array();
  if (shape.empty()) return Json(v[off++]);
  for (int64_t i = 0; i < shape[d]; ++i) {
    if (d + 1 == shape.size()) a.push_back(Json(v[off++]));
    else a.push_back(dense_to_json(shape, v, d + 1, off));
  }
  return a;
}

template <class T>
void push_all(std::vector<double>& out, const std::vector<T>& in) {
  out.reserve(out.size() + in.size());
  for (const auto& x : in) out.push_back(double(x));
}

double half_to_double(uint16_t h) {
  uint32_t sign = (h >> 15) & 1, exp = (h >> 10) & 0x1F, mant = h & 0x3FF;
  double v;
  if (exp == 0) v = std::ldexp(double(mant), -24);
  else if (exp == 31) v = mant ? NAN : INFINITY;
  else v = std::ldexp(double(mant | 0x400), int(exp) - 25);
  return sign ? -v : v;
}

}  // namespace

bool TfTensor::to_dense(std::vector<int64_t>& shape, std::vector<double>& v, std::string* err) const {
  shape = dims;
  int64_t n = 1;
  for (auto d : dims) {
    if (d < 0) {
      if (err) *err = "negative dimension in tftensor shape";
      return false;
    }
    n *= d;
  }
  v.clear();
  if (!content.empty()) {
    const char* p = content.data();
    size_t bytes = content.size();
    auto need = [&](size_t esz) {
      if (bytes != size_t(n) * esz) {
        if (err) *err = "tftensor content size does not match shape";
        return false;
      }
      return true;
    };
    v.resize(size_t(n));
    switch (dtype) {
      case DT_FLOAT: { if (!need(4)) return false; for (int64_t i = 0; i < n; ++i) { float f; memcpy(&f, p + 4 * i, 4); v[i] = f; } return true; }
      case DT_DOUBLE: { if (!need(8)) return false; if (n > 0) memcpy(v.data(), p, 8 * n); return true; }
      case DT_INT32: { if (!need(4)) return false; for (int64_t i = 0; i < n; ++i) { int32_t x; memcpy(&x, p + 4 * i, 4); v[i] = x; } return true; }
      case DT_INT64: { if (!need(8)) return false; for (int64_t i = 0; i < n; ++i) { int64_t x; memcpy(&x, p + 8 * i, 8); v[i] = double(x); } return true; }
      case DT_INT16: { if (!need(2)) return false; for (int64_t i = 0; i < n; ++i) { int16_t x; memcpy(&x, p + 2 * i, 2); v[i] = x; } return true; }
      case DT_UINT16: { if (!need(2)) return false; for (int64_t i = 0; i < n; ++i) { uint16_t x; memcpy(&x, p + 2 * i, 2); v[i] = x; } return true; }
      case DT_INT8: { if (!need(1)) return false; for (int64_t i = 0; i < n; ++i) v[i] = double(int8_t(p[i])); return true; }
      case DT_UINT8: case DT_BOOL: { if (!need(1)) return false; for (int64_t i = 0; i < n; ++i) v[i] = double(uint8_t(p[i])); return true; }
      case DT_HALF: { if (!need(2)) return false; for (int64_t i = 0; i < n; ++i) { uint16_t x; memcpy(&x, p + 2 * i, 2); v[i] = half_to_double(x); } return true; }
      case DT_UINT32: { if (!need(4)) return false; for (int64_t i = 0; i < n; ++i) { uint32_t x; memcpy(&x, p + 4 * i, 4); v[i] = x; } return true; }
      case DT_UINT64: { if (!need(8)) return false; for (int64_t i = 0; i < n; ++i) { uint64_t x; memcpy(&x, p + 8 * i, 8); v[i] = double(x); } return true; }
      default:
        if (err) *err = std::string("unsupported tftensor dtype ") + tf_dtype_name(dtype);
        return false;
    }
  }
  std::vector<double> src;
  switch (dtype) {
    case DT_FLOAT: push_all(src, float_val); break;
    case DT_DOUBLE: push_all(src, double_val); break;
    case DT_INT32: case DT_INT16: case DT_INT8: case DT_UINT8: case DT_UINT16: push_all(src, int_val); break;
    case DT_INT64: push_all(src, int64_val); break;
    case DT_BOOL: push_all(src, bool_val); break;
    case DT_UINT32: push_all(src, uint32_val); break;
    case DT_UINT64: push_all(src, uint64_val); break;
    case DT_HALF: case DT_BFLOAT16:
      for (int32_t h : half_val) src.push_back(dtype == DT_HALF ? half_to_double(uint16_t(h)) : [&] { uint32_t b = uint32_t(h) << 16; float f; memcpy(&f, &b, 4); return double(f); }());
      break;
    default:
      if (err) *err = std::string("unsupported tftensor dtype ") + tf_dtype_name(dtype);
      return false;
  }
  if (int64_t(src.size()) == n) { v = std::move(src); return true; }
  if (src.size() == 1 || (src.empty() && n > 0)) {  // TF broadcasts the last element
    double fill = src.empty() ? 0.0 : src[0];
    v.assign(size_t(n), fill);
    return true;
  }
  if (err) *err = "tftensor value count does not match shape";
  return false;
}

TfTensor TfTensor::from_dense(const std::vector<int64_t>& shape, const double* v, size_t n) {
  TfTensor t;
  t.dtype = DT_DOUBLE;
  t.dims = shape;
  t.content.assign(reinterpret_cast<const char*>(v), n * sizeof(double));
  return t;
}

bool DefaultData::dense(std::vector<int64_t>& shp, std::vector<double>& vals, std::string* err) const {
  shp.clear();
  vals.clear();
  switch (kind) {
    case DataKind::Tensor: {
      shp = shape;
      int64_t n = 1;
      for (auto d : shape) {
        if (d < 0) {
          if (err) *err = "negative dimension in tensor shape";
          return false;
        }
        n *= d;
      }
      if (n != int64_t(values.size())) {
        if (err) *err = "tensor values do not match shape";
        return false;
      }
      vals = values;
      return true;
    }
    case DataKind::NdArray:
      if (nd_dense) { shp = shape; vals = values; return true; }
      json_shape(ndarray, shp);
      vals.reserve(64);
      return json_fill(ndarray, shp, 0, vals, err);
    case DataKind::TfTensor:
      return tftensor.to_dense(shp, vals, err);
    case DataKind::None:
      return true;
  }
  return false;
}

void DefaultData::set_dense(DataKind k, std::vector<int64_t> shp, std::vector<double> vals) {
  kind = k == DataKind::None ? DataKind::Tensor : k;
  ndarray = Json();
  nd_dense = false;
  tftensor = TfTensor();
  if (kind == DataKind::TfTensor) {
    tftensor = TfTensor::from_dense(shp, vals.data(), vals.size());
    shape.clear();
    values.clear();
    return;
  }
  nd_dense = (kind == DataKind::NdArray);
  shape = std::move(shp);
  values = std::move(vals);
}

int64_t DefaultData::rows() const {
  switch (kind) {
    case DataKind::Tensor: return shape.empty() ? 0 : shape[0];
    case DataKind::NdArray: return nd_dense ? (shape.empty() ? 0 : shape[0]) : int64_t(ndarray.size());
    case DataKind::TfTensor: return tftensor.dims.empty() ? 0 : tftensor.dims[0];
    default: return 0;
  }
}

// ----------------------------------------------------------------- JSON in
namespace {

[[noreturn]] void bad(const std::string& why) { throw CodecError(why); }

const Json* field(const Json& obj, const char* json_name, const char* proto_name = nullptr) {
  const Json* f = obj.find(json_name);
  if (!f && proto_name) f = obj.find(proto_name);
  if (f && f->is_null()) return nullptr;
  return f;
}

void check_known(const Json& obj, std::initializer_list<const char*> known, const char* what) {
  if (!obj.is_object()) bad(std::string("expected object for ") + what);
  for (const auto& m : obj.members()) {
    bool ok = false;
    for (const char* k : known)
      if (m.first == k) { ok = true; break; }
    if (!ok) bad("Cannot find field: " + m.first + " in message " + what);
  }
}

std::string get_str(const Json& j, const char* what) {
  if (!j.is_string()) bad(std::string("expected string for ") + what);
  return j.as_string();
}

int64_t get_int(const Json& j, const char* what) {
  if (j.is_number()) {
    double d = j.as_number();
    if (d != std::floor(d)) bad(std::string("expected integer for ") + what);
    return int64_t(d);
  }
  if (j.is_string()) {
    double d;
    const std::string& s = j.as_string();
    if (!parse_double(s.data(), s.data() + s.size(), d) || d != std::floor(d))
      bad(std::string("expected integer for ") + what);
    return int64_t(d);
  }
  bad(std::string("expected integer for ") + what);
}

double get_num(const Json& j, const char* what) {
  if (j.is_number()) return j.as_number();
  if (j.is_string()) {
    const std::string& s = j.as_string();
    if (s == "NaN") return NAN;
    if (s == "Infinity") return INFINITY;
    if (s == "-Infinity") return -INFINITY;
    double d;
    if (parse_double(s.data(), s.data() + s.size(), d)) return d;
  }
  bad(std::string("expected number for ") + what);
}

bool get_bool(const Json& j, const char* what) {
  if (j.is_bool()) return j.as_bool();
  bad(std::string("expected bool for ") + what);
}

void parse_strmap(const Json& j, StrMap& out, const char* what) {
  if (!j.is_object()) bad(std::string("expected object for ") + what);
  for (const auto& m : j.members()) {
    if (m.second.is_string()) out.emplace_back(m.first, m.second.as_string());
    else if (m.second.is_number() || m.second.is_bool()) out.emplace_back(m.first, m.second.dump());
    else bad(std::string("expected string map value in ") + what);
  }
}

void parse_metric(const Json& j, Metric& mt) {
  check_known(j, {"key", "type", "value", "tags"}, "seldon.protos.Metric");
  if (auto* f = field(j, "key")) mt.key = get_str(*f, "Metric.key");
  if (auto* f = field(j, "type")) {
    if (f->is_string()) {
      const std::string& s = f->as_string();
      if (s == "COUNTER") mt.type = MetricType::COUNTER;
      else if (s == "GAUGE") mt.type = MetricType::GAUGE;
      else if (s == "TIMER") mt.type = MetricType::TIMER;
      else bad("Invalid enum value " + s + " for enum type seldon.protos.Metric.MetricType");
    } else {
      int64_t v = get_int(*f, "Metric.type");
      if (v < 0 || v > 2) bad("Invalid metric type");
      mt.type = MetricType(v);
    }
  }
  if (auto* f = field(j, "value")) mt.value = float(get_num(*f, "Metric.value"));
  if (auto* f = field(j, "tags")) parse_strmap(*f, mt.tags, "Metric.tags");
}

void parse_meta(const Json& j, Meta& m) {
  check_known(j, {"puid", "tags", "routing", "requestPath", "request_path", "metrics"}, "seldon.protos.Meta");
  if (auto* f = field(j, "puid")) m.puid = get_str(*f, "Meta.puid");
  if (auto* f = field(j, "tags")) {
    if (!f->is_object()) bad("expected object for Meta.tags");
    for (const auto& kv : f->members()) m.put_tag(kv.first, kv.second);
  }
  if (auto* f = field(j, "routing")) {
    if (!f->is_object()) bad("expected object for Meta.routing");
    for (const auto& kv : f->members()) m.put_routing(kv.first, int32_t(get_int(kv.second, "Meta.routing")));
  }
  if (auto* f = field(j, "requestPath", "request_path")) {
    StrMap tmp;
    parse_strmap(*f, tmp, "Meta.requestPath");
    for (auto& kv : tmp) m.put_request_path(kv.first, kv.second);
  }
  if (auto* f = field(j, "metrics")) {
    if (!f->is_array()) bad("expected array for Meta.metrics");
    for (const auto& x : f->items()) {
      Metric mt;
      parse_metric(x, mt);
      m.metrics.push_back(std::move(mt));
    }
  }
}

void parse_status(const Json& j, Status& s) {
  check_known(j, {"code", "info", "reason", "status"}, "seldon.protos.Status");
  if (auto* f = field(j, "code")) s.code = int32_t(get_int(*f, "Status.code"));
  if (auto* f = field(j, "info")) s.info = get_str(*f, "Status.info");
  if (auto* f = field(j, "reason")) s.reason = get_str(*f, "Status.reason");
  if (auto* f = field(j, "status")) {
    if (f->is_string()) {
      if (f->as_string() == "SUCCESS") s.status = 0;
      else if (f->as_string() == "FAILURE") s.status = 1;
      else bad("Invalid enum value for Status.status");
    } else {
      s.status = int32_t(get_int(*f, "Status.status"));
    }
  }
}

template <class T, class F>
void parse_num_list(const Json* f, std::vector<T>& out, const char* what, F conv) {
  if (!f) return;
  if (!f->is_array()) bad(std::string("expected array for ") + what);
  out.reserve(f->items().size());
  for (const auto& x : f->items()) out.push_back(conv(x));
}

void parse_tftensor(const Json& j, TfTensor& t) {
  if (!j.is_object()) bad("expected object for tftensor");
  if (auto* f = field(j, "dtype")) {
    if (f->is_string()) {
      int32_t d = tf_dtype_from_name(f->as_string());
      if (d < 0) bad("Invalid enum value " + f->as_string() + " for enum type tensorflow.DataType");
      t.dtype = d;
    } else {
      t.dtype = int32_t(get_int(*f, "tftensor.dtype"));
    }
  }
  if (auto* f = field(j, "tensorShape", "tensor_shape")) {
    if (!f->is_object()) bad("expected object for tensorShape");
    if (auto* d = field(*f, "dim")) {
      if (!d->is_array()) bad("expected array for tensorShape.dim");
      for (const auto& x : d->items()) {
        int64_t sz = 0;
        if (auto* s = field(x, "size")) sz = get_int(*s, "dim.size");
        if (sz < 0) bad("negative dimension in tensorShape");
        t.dims.push_back(sz);
      }
    }
    if (auto* u = field(*f, "unknownRank", "unknown_rank")) t.unknown_rank = get_bool(*u, "unknownRank");
  }
  if (auto* f = field(j, "versionNumber", "version_number")) t.version_number = int32_t(get_int(*f, "versionNumber"));
  if (auto* f = field(j, "tensorContent", "tensor_content")) {
    if (!base64_decode(get_str(*f, "tensorContent"), t.content)) bad("invalid base64 in tensorContent");
  }
  auto num = [](const Json& x) { return get_num(x, "tftensor value"); };
  auto integer = [](const Json& x) { return get_int(x, "tftensor value"); };
  parse_num_list(field(j, "floatVal", "float_val"), t.float_val, "floatVal", [&](const Json& x) { return float(num(x)); });
  parse_num_list(field(j, "doubleVal", "double_val"), t.double_val, "doubleVal", num);
  parse_num_list(field(j, "intVal", "int_val"), t.int_val, "intVal", [&](const Json& x) { return int32_t(integer(x)); });
  parse_num_list(field(j, "int64Val", "int64_val"), t.int64_val, "int64Val", integer);
  parse_num_list(field(j, "halfVal", "half_val"), t.half_val, "halfVal", [&](const Json& x) { return int32_t(integer(x)); });
  parse_num_list(field(j, "scomplexVal", "scomplex_val"), t.scomplex_val, "scomplexVal", [&](const Json& x) { return float(num(x)); });
  parse_num_list(field(j, "dcomplexVal", "dcomplex_val"), t.dcomplex_val, "dcomplexVal", num);
  parse_num_list(field(j, "uint32Val", "uint32_val"), t.uint32_val, "uint32Val", [&](const Json& x) { return uint32_t(integer(x)); });
  parse_num_list(field(j, "uint64Val", "uint64_val"), t.uint64_val, "uint64Val", [&](const Json& x) { return uint64_t(integer(x)); });
  parse_num_list(field(j, "boolVal", "bool_val"), t.bool_val, "boolVal", [](const Json& x) { return uint8_t(get_bool(x, "boolVal")); });
  if (auto* f = field(j, "stringVal", "string_val")) {
    if (!f->is_array()) bad("expected array for stringVal");
    for (const auto& x : f->items()) {
      std::string raw;
      if (!base64_decode(get_str(x, "stringVal"), raw)) bad("invalid base64 in stringVal");
      t.string_val.push_back(std::move(raw));
    }
  }
}

void parse_default_data(const Json& j, DefaultData& d) {
  check_known(j, {"names", "tensor", "ndarray", "tftensor"}, "seldon.protos.DefaultData");
  if (auto* f = field(j, "names")) {
    if (!f->is_array()) bad("expected array for DefaultData.names");
    for (const auto& x : f->items()) d.names.push_back(get_str(x, "DefaultData.names"));
  }
  int set = 0;
  if (auto* f = field(j, "tensor")) {
    ++set;
    d.kind = DataKind::Tensor;
    check_known(*f, {"shape", "values"}, "seldon.protos.Tensor");
    if (auto* s = field(*f, "shape")) {
      if (!s->is_array()) bad("expected array for Tensor.shape");
      for (const auto& x : s->items()) {
        int64_t dim = get_int(x, "Tensor.shape");
        if (dim < 0) bad("negative dimension in Tensor.shape");
        d.shape.push_back(dim);
      }
    }
    if (auto* v = field(*f, "values")) {
      if (!v->is_array()) bad("expected array for Tensor.values");
      d.values.reserve(v->items().size());
      for (const auto& x : v->items()) d.values.push_back(get_num(x, "Tensor.values"));
    }
  }
  if (auto* f = field(j, "ndarray")) {
    ++set;
    if (!f->is_array()) bad("expected array for DefaultData.ndarray");
    d.kind = DataKind::NdArray;
    d.ndarray = *f;
  }
  if (auto* f = field(j, "tftensor")) {
    ++set;
    d.kind = DataKind::TfTensor;
    parse_tftensor(*f, d.tftensor);
  }
  if (set > 1) bad("Message type \"seldon.protos.DefaultData\" has more than one field set in oneof \"data_oneof\"");
}

}  // namespace

void message_from_json(const Json& j, SeldonMessage& m) {
  check_known(j, {"status", "meta", "data", "binData", "bin_data", "strData", "str_data", "jsonData", "json_data"},
              "seldon.protos.SeldonMessage");
  if (auto* f = field(j, "status")) { m.has_status = true; parse_status(*f, m.status); }
  if (auto* f = field(j, "meta")) { m.has_meta = true; parse_meta(*f, m.meta); }
  int set = 0;
  if (auto* f = field(j, "data")) { ++set; m.payload = Payload::Data; parse_default_data(*f, m.data); }
  if (auto* f = field(j, "binData", "bin_data")) {
    ++set;
    m.payload = Payload::BinData;
    if (!base64_decode(get_str(*f, "binData"), m.bin_data)) bad("invalid base64 in binData");
  }
  if (auto* f = field(j, "strData", "str_data")) { ++set; m.payload = Payload::StrData; m.str_data = get_str(*f, "strData"); }
  if (const Json* f = j.find("jsonData") ? j.find("jsonData") : j.find("json_data")) {
    ++set;
    m.payload = Payload::JsonData;
    m.json_data = *f;
  }
  if (set > 1) bad("Message type \"seldon.protos.SeldonMessage\" has more than one field set in oneof \"data_oneof\"");
}

bool fast_dense_message(std::string_view text, SeldonMessage& m) {
  const char* p = text.data();
  const char* const e = p + text.size();
  auto ws = [&] {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  };
  auto lit = [&](char c) {
    ws();
    if (p < e && *p == c) { ++p; return true; }
    return false;
  };
  auto str = [&](std::string_view& out) {  // plain string: no escapes / control characters
    ws();
    if (p >= e || *p != '"') return false;
    const char* b = ++p;
    while (p < e && *p != '"') {
      if (*p == '\\' || static_cast<unsigned char>(*p) < 0x20) return false;
      ++p;
    }
    if (p >= e) return false;
    out = std::string_view(b, size_t(p - b));
    ++p;
    return true;
  };
  auto number = [&](double& d) {  // the general parser's token rule, then the same conversion
    ws();
    const char* b = p;
    if (p < e && *p == '-') ++p;
    while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) ++p;
    return p != b && parse_double(b, p, d);
  };
  std::vector<std::string> names;
  std::vector<double> vals;
  int64_t rows = 0, cols = -1;
  bool have_data = false, have_meta = false, have_names = false, have_nd = false;
  if (!lit('{')) return false;
  for (;;) {
    std::string_view k;
    if (!str(k) || !lit(':')) return false;
    if (k == "data" && !have_data) {
      have_data = true;
      if (!lit('{')) return false;
      for (;;) {
        std::string_view dk;
        if (!str(dk) || !lit(':')) return false;
        if (dk == "names" && !have_names) {
          have_names = true;
          if (!lit('[')) return false;
          if (!lit(']')) {
            for (;;) {
              std::string_view nm;
              if (!str(nm)) return false;
              names.emplace_back(nm);
              if (lit(',')) continue;
              if (lit(']')) break;
              return false;
            }
          }
        } else if (dk == "ndarray" && !have_nd) {
          have_nd = true;
          if (!lit('[')) return false;
          for (;;) {
            if (!lit('[')) return false;
            int64_t c = 0;
            for (;;) {
              double d;
              if (!number(d)) return false;
              vals.push_back(d);
              ++c;
              if (lit(',')) continue;
              if (lit(']')) break;
              return false;
            }
            if (cols < 0) cols = c;
            else if (c != cols) return false;
            ++rows;
            if (lit(',')) continue;
            if (lit(']')) break;
            return false;
          }
        } else {
          return false;
        }
        if (lit(',')) continue;
        if (lit('}')) break;
        return false;
      }
    } else if (k == "meta" && !have_meta) {
      have_meta = true;
      if (!lit('{') || !lit('}')) return false;
    } else {
      return false;
    }
    if (lit(',')) continue;
    if (lit('}')) break;
    return false;
  }
  ws();
  if (p != e || !have_nd) return false;
  m.payload = Payload::Data;
  if (have_meta) m.has_meta = true;
  m.data.names = std::move(names);
  m.data.set_dense(DataKind::NdArray, {rows, cols}, std::move(vals));
  return true;
}

void feedback_from_json(const Json& j, Feedback& f) {
  check_known(j, {"request", "response", "reward", "truth"}, "seldon.protos.Feedback");
  if (auto* x = field(j, "request")) { f.has_request = true; message_from_json(*x, f.request); }
  if (auto* x = field(j, "response")) { f.has_response = true; message_from_json(*x, f.response); }
  if (auto* x = field(j, "truth")) { f.has_truth = true; message_from_json(*x, f.truth); }
  if (auto* x = field(j, "reward")) f.reward = float(get_num(*x, "Feedback.reward"));
}

void message_list_from_json(const Json& j, std::vector<SeldonMessage>& out) {
  check_known(j, {"seldonMessages", "seldon_messages"}, "seldon.protos.SeldonMessageList");
  if (auto* f = field(j, "seldonMessages", "seldon_messages")) {
    if (!f->is_array()) bad("expected array for seldonMessages");
    for (const auto& x : f->items()) {
      out.emplace_back();
      message_from_json(x, out.back());
    }
  }
}

// ---------------------------------------------------------------- JSON out
namespace {

void write_strmap(std::string& out, const StrMap& m) {
  out.push_back('{');
  bool first = true;
  for (const auto& kv : m) {
    if (!first) out.push_back(',');
    first = false;
    append_quoted(out, kv.first);
    out.push_back(':');
    append_quoted(out, kv.second);
  }
  out.push_back('}');
}

void write_meta(std::string& out, const Meta& m) {
  out += "{\"puid\":";
  append_quoted(out, m.puid);
  out += ",\"tags\":{";
  bool first = true;
  for (const auto& kv : m.tags) {
    if (!first) out.push_back(',');
    first = false;
    append_quoted(out, kv.first);
    out.push_back(':');
    write_json(kv.second, out);
  }
  out += "},\"routing\":{";
  first = true;
  for (const auto& kv : m.routing) {
    if (!first) out.push_back(',');
    first = false;
    append_quoted(out, kv.first);
    out.push_back(':');
    out += std::to_string(kv.second);
  }
  out += "},\"requestPath\":";
  write_strmap(out, m.request_path);
  out += ",\"metrics\":[";
  first = true;
  for (const auto& mt : m.metrics) {
    if (!first) out.push_back(',');
    first = false;
    out += "{\"key\":";
    append_quoted(out, mt.key);
    out += ",\"type\":\"";
    out += metric_type_name(mt.type);
    out += "\",\"value\":";
    append_float(out, mt.value);
    out += ",\"tags\":";
    write_strmap(out, mt.tags);
    out.push_back('}');
  }
  out += "]}";
}

void write_i64_str_list(std::string& out, const std::vector<int64_t>& v) {
  out.push_back('[');
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out.push_back(',');
    out.push_back('"');
    out += std::to_string(v[i]);
    out.push_back('"');
  }
  out.push_back(']');
}

template <class T>
void write_num_list(std::string& out, const char* name, const std::vector<T>& v, bool& first) {
  if (v.empty()) return;
  if (!first) out.push_back(',');
  first = false;
  out.push_back('"');
  out += name;
  out += "\":[";
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out.push_back(',');
    if constexpr (std::is_floating_point_v<T>) {
      if constexpr (std::is_same_v<T, float>) append_float(out, v[i]);
      else append_number(out, v[i]);
    } else if constexpr (std::is_same_v<T, uint8_t>) {
      out += v[i] ? "true" : "false";
    } else if constexpr (sizeof(T) == 8) {
      out.push_back('"');
      out += std::to_string(v[i]);
      out.push_back('"');
    } else {
      out += std::to_string(v[i]);
    }
  }
  out.push_back(']');
}

void write_tftensor(std::string& out, const TfTensor& t) {
  out += "{\"dtype\":\"";
  out += tf_dtype_name(t.dtype);
  out += "\",\"tensorShape\":{\"dim\":[";
  for (size_t i = 0; i < t.dims.size(); ++i) {
    if (i) out.push_back(',');
    out += "{\"size\":\"";
    out += std::to_string(t.dims[i]);
    out += "\"}";
  }
  out += "]";
  if (t.unknown_rank) out += ",\"unknownRank\":true";
  out += "}";
  bool first = false;
  if (t.version_number) { out += ",\"versionNumber\":"; out += std::to_string(t.version_number); }
  if (!t.content.empty()) {
    out += ",\"tensorContent\":";
    append_quoted(out, base64_encode(t.content));
  }
  write_num_list(out, "floatVal", t.float_val, first);
  write_num_list(out, "doubleVal", t.double_val, first);
  write_num_list(out, "intVal", t.int_val, first);
  if (!t.string_val.empty()) {
    out += ",\"stringVal\":[";
    for (size_t i = 0; i < t.string_val.size(); ++i) {
      if (i) out.push_back(',');
      append_quoted(out, base64_encode(t.string_val[i]));
    }
    out.push_back(']');
  }
  write_num_list(out, "scomplexVal", t.scomplex_val, first);
  write_num_list(out, "int64Val", t.int64_val, first);
  write_num_list(out, "boolVal", t.bool_val, first);
  write_num_list(out, "dcomplexVal", t.dcomplex_val, first);
  write_num_list(out, "halfVal", t.half_val, first);
  write_num_list(out, "uint32Val", t.uint32_val, first);
  write_num_list(out, "uint64Val", t.uint64_val, first);
  out.push_back('}');
}

void write_default_data(std::string& out, const DefaultData& d) {
  out += "{\"names\":[";
  for (size_t i = 0; i < d.names.size(); ++i) {
    if (i) out.push_back(',');
    append_quoted(out, d.names[i]);
  }
  out.push_back(']');
  switch (d.kind) {
    case DataKind::Tensor: {
      out += ",\"tensor\":{\"shape\":[";
      for (size_t i = 0; i < d.shape.size(); ++i) {
        if (i) out.push_back(',');
        out += std::to_string(d.shape[i]);
      }
      out += "],\"values\":[";
      for (size_t i = 0; i < d.values.size(); ++i) {
        if (i) out.push_back(',');
        append_number(out, d.values[i]);
      }
      out += "]}";
      break;
    }
    case DataKind::NdArray:
      out += ",\"ndarray\":";
      if (d.nd_dense) {
        size_t off = 0;
        if (d.shape.empty()) out += "[]";
        else write_dense_nd(out, d.shape, d.values.data(), 0, off);
      } else {
        write_json(d.ndarray, out);
      }
      break;
    case DataKind::TfTensor:
      out += ",\"tftensor\":";
      write_tftensor(out, d.tftensor);
      break;
    case DataKind::None:
      break;
  }
  out.push_back('}');
}

}  // namespace

void status_to_json(const Status& s, std::string& out) {
  out += "{\"code\":";
  out += std::to_string(s.code);
  out += ",\"info\":";
  append_quoted(out, s.info);
  out += ",\"reason\":";
  append_quoted(out, s.reason);
  out += s.status ? ",\"status\":\"FAILURE\"}" : ",\"status\":\"SUCCESS\"}";
}

void message_to_json(const SeldonMessage& m, std::string& out) {
  out.push_back('{');
  bool first = true;
  auto sep = [&] { if (!first) out.push_back(','); first = false; };
  if (m.has_status) { sep(); out += "\"status\":"; status_to_json(m.status, out); }
  if (m.has_meta) { sep(); out += "\"meta\":"; write_meta(out, m.meta); }
  switch (m.payload) {
    case Payload::Data: sep(); out += "\"data\":"; write_default_data(out, m.data); break;
    case Payload::BinData: sep(); out += "\"binData\":"; append_quoted(out, base64_encode(m.bin_data)); break;
    case Payload::StrData: sep(); out += "\"strData\":"; append_quoted(out, m.str_data); break;
    case Payload::JsonData: sep(); out += "\"jsonData\":"; write_json(m.json_data, out); break;
    case Payload::None: break;
  }
  out.push_back('}');
}

Json message_to_json_value(const SeldonMessage& m) {
  std::string s;
  message_to_json(m, s);
  return parse_json(s);
}

void feedback_to_json(const Feedback& f, std::string& out) {
  out.push_back('{');
  bool first = true;
  auto sep = [&] { if (!first) out.push_back(','); first = false; };
  if (f.has_request) { sep(); out += "\"request\":"; message_to_json(f.request, out); }
  if (f.has_response) { sep(); out += "\"response\":"; message_to_json(f.response, out); }
  sep();
  out += "\"reward\":";
  append_float(out, f.reward);
  if (f.has_truth) { sep(); out += "\"truth\":"; message_to_json(f.truth, out); }
  out.push_back('}');
}

void message_list_to_json(const std::vector<const SeldonMessage*>& msgs, std::string& out) {
  out += "{\"seldonMessages\":[";
  for (size_t i = 0; i < msgs.size(); ++i) {
    if (i) out.push_back(',');
    message_to_json(*msgs[i], out);
  }
  out += "]}";
}

}  // namespace sca
