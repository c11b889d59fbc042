// Hand-rolled protobuf wire codec for prediction.proto.
//
// The reference relies on generated stubs (protobuf-java in the engine,
// prediction_pb2 in Python).  The MI355X engine decodes gRPC
// payloads directly into the C++ message struct so the packed
// `Tensor.values` doubles are memcpy'd into the dense buffer that is later
// staged to the GPU (cf. the np.frombuffer trick at
// python/seldon_core/utils.py:163-169).
#include <cstring>

#include "message.h"

namespace sca {
namespace {

// ------------------------------------------------------------------ writer
inline void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(char(v | 0x80));
    v >>= 7;
  }
  o.push_back(char(v));
}
inline void put_tag(std::string& o, uint32_t field, uint32_t wt) { put_varint(o, (uint64_t(field) << 3) | wt); }
inline void put_bytes(std::string& o, uint32_t field, std::string_view s) {
  put_tag(o, field, 2);
  put_varint(o, s.size());
  o.append(s.data(), s.size());
}
inline void put_str_nonempty(std::string& o, uint32_t field, std::string_view s) {
  if (!s.empty()) put_bytes(o, field, s);
}
inline void put_int32(std::string& o, uint32_t field, int32_t v) {
  if (!v) return;
  put_tag(o, field, 0);
  put_varint(o, uint64_t(int64_t(v)));
}
inline void put_double(std::string& o, uint32_t field, double v) {
  put_tag(o, field, 1);
  char b[8];
  memcpy(b, &v, 8);
  o.append(b, 8);
}
inline void put_float(std::string& o, uint32_t field, float v) {
  put_tag(o, field, 5);
  char b[4];
  memcpy(b, &v, 4);
  o.append(b, 4);
}

void enc_value(std::string& o, const Json& v);

void enc_list(std::string& o, const Json& a) {  // ListValue body
  for (const auto& x : a.items()) {
    std::string sub;
    enc_value(sub, x);
    put_bytes(o, 1, sub);
  }
}

void enc_struct(std::string& o, const Json& obj) {  // Struct body
  for (const auto& kv : obj.members()) {
    std::string entry, val;
    put_bytes(entry, 1, kv.first);
    enc_value(val, kv.second);
    put_bytes(entry, 2, val);
    put_bytes(o, 1, entry);
  }
}

void enc_value(std::string& o, const Json& v) {  // google.protobuf.Value body
  switch (v.type()) {
    case Json::Type::Null: put_tag(o, 1, 0); put_varint(o, 0); break;
    case Json::Type::Number: put_double(o, 2, v.as_number()); break;
    case Json::Type::String: put_bytes(o, 3, v.as_string()); break;
    case Json::Type::Bool: put_tag(o, 4, 0); put_varint(o, v.as_bool() ? 1 : 0); break;
    case Json::Type::Object: { std::string s; enc_struct(s, v); put_bytes(o, 5, s); break; }
    case Json::Type::Array: { std::string s; enc_list(s, v); put_bytes(o, 6, s); break; }
  }
}

void enc_dense_list(std::string& o, const std::vector<int64_t>& shape, const double* v, size_t d, size_t& off) {
  // ListValue body for a dense nd block
  for (int64_t i = 0; i < shape[d]; ++i) {
    std::string val;
    if (d + 1 == shape.size()) {
      put_double(val, 2, v[off++]);
    } else {
      std::string inner;
      enc_dense_list(inner, shape, v, d + 1, off);
      put_bytes(val, 6, inner);
    }
    put_bytes(o, 1, val);
  }
}

void enc_strmap(std::string& o, uint32_t field, const StrMap& m) {
  for (const auto& kv : m) {
    std::string e;
    put_bytes(e, 1, kv.first);
    put_bytes(e, 2, kv.second);
    put_bytes(o, field, e);
  }
}

void enc_meta(std::string& o, const Meta& m) {
  put_str_nonempty(o, 1, m.puid);
  for (const auto& kv : m.tags) {
    std::string e, val;
    put_bytes(e, 1, kv.first);
    enc_value(val, kv.second);
    put_bytes(e, 2, val);
    put_bytes(o, 2, e);
  }
  for (const auto& kv : m.routing) {
    std::string e;
    put_bytes(e, 1, kv.first);
    put_tag(e, 2, 0);
    put_varint(e, uint64_t(int64_t(kv.second)));
    put_bytes(o, 3, e);
  }
  enc_strmap(o, 4, m.request_path);
  for (const auto& mt : m.metrics) {
    std::string s;
    put_str_nonempty(s, 1, mt.key);
    put_int32(s, 2, int32_t(mt.type));
    if (mt.value != 0.f) put_float(s, 3, mt.value);
    enc_strmap(s, 4, mt.tags);
    put_bytes(o, 5, s);
  }
}

void enc_status(std::string& o, const Status& s) {
  put_int32(o, 1, s.code);
  put_str_nonempty(o, 2, s.info);
  put_str_nonempty(o, 3, s.reason);
  put_int32(o, 4, s.status);
}

template <class T>
void enc_packed_fixed(std::string& o, uint32_t field, const std::vector<T>& v) {
  if (v.empty()) return;
  put_tag(o, field, 2);
  put_varint(o, v.size() * sizeof(T));
  o.append(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(T));
}
template <class T>
void enc_packed_varint(std::string& o, uint32_t field, const std::vector<T>& v) {
  if (v.empty()) return;
  std::string body;
  for (auto x : v) put_varint(body, uint64_t(int64_t(x)));
  put_bytes(o, field, body);
}

void enc_tftensor(std::string& o, const TfTensor& t) {
  put_int32(o, 1, t.dtype);
  {
    std::string shp;
    for (auto d : t.dims) {
      std::string dim;
      if (d) { put_tag(dim, 1, 0); put_varint(dim, uint64_t(d)); }
      put_bytes(shp, 2, dim);
    }
    if (t.unknown_rank) { put_tag(shp, 3, 0); put_varint(shp, 1); }
    put_bytes(o, 2, shp);
  }
  put_int32(o, 3, t.version_number);
  if (!t.content.empty()) put_bytes(o, 4, t.content);
  enc_packed_fixed(o, 5, t.float_val);
  enc_packed_fixed(o, 6, t.double_val);
  enc_packed_varint(o, 7, t.int_val);
  for (const auto& s : t.string_val) put_bytes(o, 8, s);
  enc_packed_fixed(o, 9, t.scomplex_val);
  enc_packed_varint(o, 10, t.int64_val);
  enc_packed_varint(o, 11, t.bool_val);
  enc_packed_fixed(o, 12, t.dcomplex_val);
  enc_packed_varint(o, 13, t.half_val);
  enc_packed_varint(o, 16, t.uint32_val);
  enc_packed_varint(o, 17, t.uint64_val);
}

void enc_default_data(std::string& o, const DefaultData& d) {
  for (const auto& n : d.names) put_bytes(o, 1, n);
  switch (d.kind) {
    case DataKind::Tensor: {
      std::string t;
      if (!d.shape.empty()) {
        std::string body;
        for (auto s : d.shape) put_varint(body, uint64_t(int64_t(int32_t(s))));
        put_bytes(t, 1, body);
      }
      enc_packed_fixed(t, 2, d.values);
      put_bytes(o, 2, t);
      break;
    }
    case DataKind::NdArray: {
      std::string l;
      if (d.nd_dense) {
        size_t off = 0;
        if (!d.shape.empty()) enc_dense_list(l, d.shape, d.values.data(), 0, off);
      } else {
        enc_list(l, d.ndarray);
      }
      put_bytes(o, 3, l);
      break;
    }
    case DataKind::TfTensor: {
      std::string t;
      enc_tftensor(t, d.tftensor);
      put_bytes(o, 4, t);
      break;
    }
    case DataKind::None: break;
  }
}

// ------------------------------------------------------------------ reader
struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;

  explicit Reader(std::string_view s) : p((const uint8_t*)s.data()), e((const uint8_t*)s.data() + s.size()) {}
  bool more() const { return ok && p < e; }
  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (p < e && shift < 64) {
      uint8_t b = *p++;
      v |= uint64_t(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
      shift += 7;
    }
    ok = false;
    return 0;
  }
  std::string_view bytes() {
    uint64_t n = varint();
    if (!ok || uint64_t(e - p) < n) { ok = false; return {}; }
    std::string_view s((const char*)p, size_t(n));
    p += n;
    return s;
  }
  double f64() {
    if (e - p < 8) { ok = false; return 0; }
    double d;
    memcpy(&d, p, 8);
    p += 8;
    return d;
  }
  float f32() {
    if (e - p < 4) { ok = false; return 0; }
    float f;
    memcpy(&f, p, 4);
    p += 4;
    return f;
  }
  void skip(uint32_t wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: if (e - p < 8) ok = false; else p += 8; break;
      case 2: bytes(); break;
      case 5: if (e - p < 4) ok = false; else p += 4; break;
      default: ok = false;
    }
  }
};

bool dec_value(std::string_view buf, Json& out, int depth);

bool dec_list(std::string_view buf, Json& out, int depth) {
  out = Json::array();
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    if ((tag >> 3) == 1 && (tag & 7) == 2) {
      Json v;
      if (!dec_value(r.bytes(), v, depth + 1)) return false;
      out.push_back(std::move(v));
    } else {
      r.skip(uint32_t(tag & 7));
    }
  }
  return r.ok;
}

bool dec_struct(std::string_view buf, Json& out, int depth) {
  out = Json::object();
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    if ((tag >> 3) == 1 && (tag & 7) == 2) {
      Reader er(r.bytes());
      std::string key;
      Json val;
      while (er.more()) {
        uint64_t t = er.varint();
        if ((t >> 3) == 1 && (t & 7) == 2) key = std::string(er.bytes());
        else if ((t >> 3) == 2 && (t & 7) == 2) { if (!dec_value(er.bytes(), val, depth + 1)) return false; }
        else er.skip(uint32_t(t & 7));
      }
      if (!er.ok) return false;
      out.set(key, std::move(val));
    } else {
      r.skip(uint32_t(tag & 7));
    }
  }
  return r.ok;
}

bool dec_value(std::string_view buf, Json& out, int depth) {
  if (depth > 256) return false;
  Reader r(buf);
  out = Json();
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (f == 1 && wt == 0) { r.varint(); out = Json(); }
    else if (f == 2 && wt == 1) out = Json(r.f64());
    else if (f == 3 && wt == 2) out = Json(std::string(r.bytes()));
    else if (f == 4 && wt == 0) out = Json(r.varint() != 0);
    else if (f == 5 && wt == 2) { if (!dec_struct(r.bytes(), out, depth)) return false; }
    else if (f == 6 && wt == 2) { if (!dec_list(r.bytes(), out, depth)) return false; }
    else r.skip(wt);
  }
  return r.ok;
}

void dec_strmap_entry(std::string_view buf, StrMap& m, bool& ok) {
  Reader r(buf);
  std::string k, v;
  while (r.more()) {
    uint64_t t = r.varint();
    if ((t >> 3) == 1 && (t & 7) == 2) k = std::string(r.bytes());
    else if ((t >> 3) == 2 && (t & 7) == 2) v = std::string(r.bytes());
    else r.skip(uint32_t(t & 7));
  }
  ok &= r.ok;
  m.emplace_back(std::move(k), std::move(v));
}

bool dec_meta(std::string_view buf, Meta& m) {
  Reader r(buf);
  bool ok = true;
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (f == 1 && wt == 2) m.puid = std::string(r.bytes());
    else if (f == 2 && wt == 2) {
      Reader er(r.bytes());
      std::string k;
      Json v;
      while (er.more()) {
        uint64_t t = er.varint();
        if ((t >> 3) == 1 && (t & 7) == 2) k = std::string(er.bytes());
        else if ((t >> 3) == 2 && (t & 7) == 2) { if (!dec_value(er.bytes(), v, 0)) return false; }
        else er.skip(uint32_t(t & 7));
      }
      if (!er.ok) return false;
      m.put_tag(k, std::move(v));
    } else if (f == 3 && wt == 2) {
      Reader er(r.bytes());
      std::string k;
      int32_t v = 0;
      while (er.more()) {
        uint64_t t = er.varint();
        if ((t >> 3) == 1 && (t & 7) == 2) k = std::string(er.bytes());
        else if ((t >> 3) == 2 && (t & 7) == 0) v = int32_t(er.varint());
        else er.skip(uint32_t(t & 7));
      }
      if (!er.ok) return false;
      m.put_routing(k, v);
    } else if (f == 4 && wt == 2) {
      StrMap tmp;
      dec_strmap_entry(r.bytes(), tmp, ok);
      for (auto& kv : tmp) m.put_request_path(kv.first, kv.second);
    } else if (f == 5 && wt == 2) {
      Reader mr(r.bytes());
      Metric mt;
      while (mr.more()) {
        uint64_t t = mr.varint();
        uint32_t ff = uint32_t(t >> 3), ww = uint32_t(t & 7);
        if (ff == 1 && ww == 2) mt.key = std::string(mr.bytes());
        else if (ff == 2 && ww == 0) mt.type = MetricType(int32_t(mr.varint()));
        else if (ff == 3 && ww == 5) mt.value = mr.f32();
        else if (ff == 4 && ww == 2) dec_strmap_entry(mr.bytes(), mt.tags, ok);
        else mr.skip(ww);
      }
      if (!mr.ok) return false;
      m.metrics.push_back(std::move(mt));
    } else {
      r.skip(wt);
    }
  }
  return r.ok && ok;
}

bool dec_status(std::string_view buf, Status& s) {
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (f == 1 && wt == 0) s.code = int32_t(r.varint());
    else if (f == 2 && wt == 2) s.info = std::string(r.bytes());
    else if (f == 3 && wt == 2) s.reason = std::string(r.bytes());
    else if (f == 4 && wt == 0) s.status = int32_t(r.varint());
    else r.skip(wt);
  }
  return r.ok;
}

template <class T>
void read_packed_fixed(Reader& r, uint32_t wt, std::vector<T>& out) {
  if (wt == 2) {
    std::string_view b = r.bytes();
    size_t n = b.size() / sizeof(T);
    if (n == 0) return;  // empty packed field (b.data() may be null)
    size_t old = out.size();
    out.resize(old + n);
    memcpy(out.data() + old, b.data(), n * sizeof(T));
  } else if ((sizeof(T) == 8 && wt == 1) || (sizeof(T) == 4 && wt == 5)) {
    T v;
    if (sizeof(T) == 8) { double d = r.f64(); memcpy(&v, &d, 8); }
    else { float f = r.f32(); memcpy(&v, &f, 4); }
    out.push_back(v);
  } else {
    r.skip(wt);
  }
}

template <class T>
void read_packed_varint(Reader& r, uint32_t wt, std::vector<T>& out) {
  if (wt == 2) {
    Reader pr(r.bytes());
    while (pr.more()) out.push_back(T(pr.varint()));
    r.ok &= pr.ok;
  } else if (wt == 0) {
    out.push_back(T(r.varint()));
  } else {
    r.skip(wt);
  }
}

bool dec_tftensor(std::string_view buf, TfTensor& t) {
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    switch (f) {
      case 1: if (wt == 0) t.dtype = int32_t(r.varint()); else r.skip(wt); break;
      case 2:
        if (wt == 2) {
          Reader sr(r.bytes());
          while (sr.more()) {
            uint64_t st = sr.varint();
            if ((st >> 3) == 2 && (st & 7) == 2) {
              Reader dr(sr.bytes());
              int64_t size = 0;
              while (dr.more()) {
                uint64_t dt = dr.varint();
                if ((dt >> 3) == 1 && (dt & 7) == 0) size = int64_t(dr.varint());
                else dr.skip(uint32_t(dt & 7));
              }
              if (size < 0) { sr.ok = false; break; }
              t.dims.push_back(size);
            } else if ((st >> 3) == 3 && (st & 7) == 0) {
              t.unknown_rank = sr.varint() != 0;
            } else {
              sr.skip(uint32_t(st & 7));
            }
          }
          r.ok &= sr.ok;
        } else r.skip(wt);
        break;
      case 3: if (wt == 0) t.version_number = int32_t(r.varint()); else r.skip(wt); break;
      case 4: if (wt == 2) t.content = std::string(r.bytes()); else r.skip(wt); break;
      case 5: read_packed_fixed(r, wt, t.float_val); break;
      case 6: read_packed_fixed(r, wt, t.double_val); break;
      case 7: read_packed_varint(r, wt, t.int_val); break;
      case 8: if (wt == 2) t.string_val.emplace_back(r.bytes()); else r.skip(wt); break;
      case 9: read_packed_fixed(r, wt, t.scomplex_val); break;
      case 10: read_packed_varint(r, wt, t.int64_val); break;
      case 11: read_packed_varint(r, wt, t.bool_val); break;
      case 12: read_packed_fixed(r, wt, t.dcomplex_val); break;
      case 13: read_packed_varint(r, wt, t.half_val); break;
      case 16: read_packed_varint(r, wt, t.uint32_val); break;
      case 17: read_packed_varint(r, wt, t.uint64_val); break;
      default: r.skip(wt);
    }
  }
  return r.ok;
}

bool dec_default_data(std::string_view buf, DefaultData& d) {
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (f == 1 && wt == 2) d.names.emplace_back(r.bytes());
    else if (f == 2 && wt == 2) {
      d.kind = DataKind::Tensor;
      Reader tr(r.bytes());
      while (tr.more()) {
        uint64_t t = tr.varint();
        uint32_t ff = uint32_t(t >> 3), ww = uint32_t(t & 7);
        if (ff == 1) {
          std::vector<int32_t> s;
          read_packed_varint(tr, ww, s);
          for (auto x : s) {
            if (x < 0) return false;  // numpy rejects negative dims
            d.shape.push_back(x);
          }
        } else if (ff == 2) {
          read_packed_fixed(tr, ww, d.values);
        } else {
          tr.skip(ww);
        }
      }
      if (!tr.ok) return false;
    } else if (f == 3 && wt == 2) {
      d.kind = DataKind::NdArray;
      if (!dec_list(r.bytes(), d.ndarray, 0)) return false;
    } else if (f == 4 && wt == 2) {
      d.kind = DataKind::TfTensor;
      if (!dec_tftensor(r.bytes(), d.tftensor)) return false;
    } else {
      r.skip(wt);
    }
  }
  return r.ok;
}

}  // namespace

// ------------------------------------------------------------------ public
void message_to_pb(const SeldonMessage& m, std::string& o) {
  if (m.has_status) { std::string s; enc_status(s, m.status); put_bytes(o, 1, s); }
  if (m.has_meta) { std::string s; enc_meta(s, m.meta); put_bytes(o, 2, s); }
  switch (m.payload) {
    case Payload::Data: { std::string s; enc_default_data(s, m.data); put_bytes(o, 3, s); break; }
    case Payload::BinData: put_bytes(o, 4, m.bin_data); break;
    case Payload::StrData: put_bytes(o, 5, m.str_data); break;
    case Payload::JsonData: { std::string s; enc_value(s, m.json_data); put_bytes(o, 6, s); break; }
    case Payload::None: break;
  }
}

bool message_from_pb(std::string_view buf, SeldonMessage& m) {
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (wt != 2) { r.skip(wt); continue; }
    std::string_view b = r.bytes();
    if (!r.ok) return false;
    switch (f) {
      case 1: m.has_status = true; if (!dec_status(b, m.status)) return false; break;
      case 2: m.has_meta = true; if (!dec_meta(b, m.meta)) return false; break;
      case 3: m.payload = Payload::Data; m.data = DefaultData(); if (!dec_default_data(b, m.data)) return false; break;
      case 4: m.payload = Payload::BinData; m.bin_data = std::string(b); break;
      case 5: m.payload = Payload::StrData; m.str_data = std::string(b); break;
      case 6: m.payload = Payload::JsonData; if (!dec_value(b, m.json_data, 0)) return false; break;
      default: break;
    }
  }
  return r.ok;
}

void feedback_to_pb(const Feedback& f, std::string& o) {
  if (f.has_request) { std::string s; message_to_pb(f.request, s); put_bytes(o, 1, s); }
  if (f.has_response) { std::string s; message_to_pb(f.response, s); put_bytes(o, 2, s); }
  if (f.reward != 0.f) put_float(o, 3, f.reward);
  if (f.has_truth) { std::string s; message_to_pb(f.truth, s); put_bytes(o, 4, s); }
}

bool feedback_from_pb(std::string_view buf, Feedback& fb) {
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (f == 3 && wt == 5) { fb.reward = r.f32(); continue; }
    if (wt != 2) { r.skip(wt); continue; }
    std::string_view b = r.bytes();
    if (!r.ok) return false;
    if (f == 1) { fb.has_request = true; if (!message_from_pb(b, fb.request)) return false; }
    else if (f == 2) { fb.has_response = true; if (!message_from_pb(b, fb.response)) return false; }
    else if (f == 4) { fb.has_truth = true; if (!message_from_pb(b, fb.truth)) return false; }
  }
  return r.ok;
}

void message_list_to_pb(const std::vector<const SeldonMessage*>& msgs, std::string& o) {
  for (const auto* m : msgs) {
    std::string s;
    message_to_pb(*m, s);
    put_bytes(o, 1, s);
  }
}

bool message_list_from_pb(std::string_view buf, std::vector<SeldonMessage>& out) {
  Reader r(buf);
  while (r.more()) {
    uint64_t tag = r.varint();
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (f == 1 && wt == 2) {
      out.emplace_back();
      if (!message_from_pb(r.bytes(), out.back())) return false;
    } else {
      r.skip(wt);
    }
  }
  return r.ok;
}

}  // namespace sca
