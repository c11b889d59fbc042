#include "spec.h"

#include <cstdlib>
#include <stdexcept>

namespace sca {

namespace {
const char* kTypeNames[] = {"UNKNOWN_TYPE", "ROUTER", "COMBINER", "MODEL", "TRANSFORMER", "OUTPUT_TRANSFORMER"};
const char* kImplNames[] = {"UNKNOWN_IMPLEMENTATION", "SIMPLE_MODEL", "SIMPLE_ROUTER", "RANDOM_ABTEST",
                            "AVERAGE_COMBINER", "SKLEARN_SERVER", "XGBOOST_SERVER", "TENSORFLOW_SERVER",
                            "MLFLOW_SERVER"};
const char* kMethodNames[] = {"TRANSFORM_INPUT", "TRANSFORM_OUTPUT", "ROUTE", "AGGREGATE", "SEND_FEEDBACK"};

template <size_t N>
bool lookup(const char* (&names)[N], const Json& j, int& out) {
  if (j.is_number()) {
    int v = int(j.as_number());
    if (v < 0 || v >= int(N)) return false;
    out = v;
    return true;
  }
  if (!j.is_string()) return false;
  for (size_t i = 0; i < N; ++i)
    if (j.as_string() == names[i]) { out = int(i); return true; }
  return false;
}

std::string str_of(const Json* j) {
  if (!j || j->is_null()) return "";
  if (j->is_string()) return j->as_string();
  if (j->is_number()) {
    double d = j->as_number();
    if (d == double(int64_t(d))) return std::to_string(int64_t(d));
    return j->dump();
  }
  if (j->is_bool()) return j->as_bool() ? "true" : "false";
  return j->dump();
}

const Json* field2(const Json& o, const char* a, const char* b) {
  const Json* f = o.find(a);
  if (!f) f = o.find(b);
  return f;
}

Json typed_param(const Parameter& p) {
  auto num = [&](bool integer) -> Json {
    char* end = nullptr;
    const char* s = p.value.c_str();
    double d = strtod(s, &end);
    if (end == s || *end != 0) throw std::runtime_error("Invalid value '" + p.value + "' for parameter " + p.name);
    if (integer) {
      long long v = strtoll(s, &end, 10);
      if (*end != 0) throw std::runtime_error("Invalid INT value '" + p.value + "' for parameter " + p.name);
      return Json(double(v));
    }
    return Json(d);
  };
  switch (p.type) {
    case ParamType::INT: return num(true);
    case ParamType::FLOAT: return Json(double(float(num(false).as_number())));
    case ParamType::DOUBLE: return num(false);
    case ParamType::BOOL: {
      std::string v = p.value;
      for (auto& c : v) c = char(tolower(c));
      return Json(v == "true" || v == "1");
    }
    case ParamType::STRING: default: return Json(p.value);
  }
}

void parse_unit(const Json& j, UnitSpec& u, const std::map<std::string, std::string>& images) {
  if (!j.is_object()) throw std::runtime_error("graph node must be an object");
  u.name = str_of(j.find("name"));
  if (u.name.empty()) throw std::runtime_error("graph node without a name");
  if (const Json* t = j.find("type"); t && !t->is_null()) {
    int v;
    if (!lookup(kTypeNames, *t, v)) throw std::runtime_error("Invalid type for node " + u.name + ": " + t->dump());
    u.type = UnitType(v);
    u.has_type = true;
  }
  if (const Json* t = j.find("implementation"); t && !t->is_null()) {
    int v;
    u.implementation_name = str_of(t);
    if (lookup(kImplNames, *t, v)) u.implementation = UnitImpl(v);
    else u.implementation = UnitImpl::UNKNOWN_IMPLEMENTATION;  // engine-native extension names
  }
  if (const Json* ms = j.find("methods"); ms && ms->is_array()) {
    for (const auto& m : ms->items()) {
      int v;
      if (!lookup(kMethodNames, m, v)) throw std::runtime_error("Invalid method for node " + u.name + ": " + m.dump());
      u.methods.push_back(Method(v));
    }
  }
  if (const Json* ep = j.find("endpoint"); ep && ep->is_object()) {
    u.service_host = str_of(field2(*ep, "service_host", "serviceHost"));
    std::string port = str_of(field2(*ep, "service_port", "servicePort"));
    u.service_port = port.empty() ? 0 : atoi(port.c_str());
    if (const Json* t = ep->find("type"); t && !t->is_null()) {
      if ((t->is_string() && t->as_string() == "GRPC") || (t->is_number() && t->as_number() == 1))
        u.endpoint_type = EndpointType::GRPC;
    }
  }
  if (const Json* ps = j.find("parameters"); ps && ps->is_array()) {
    for (const auto& pj : ps->items()) {
      Parameter p;
      p.name = str_of(pj.find("name"));
      p.value = str_of(pj.find("value"));
      if (const Json* t = pj.find("type"); t && !t->is_null()) {
        static const char* kPT[] = {"INT", "FLOAT", "DOUBLE", "STRING", "BOOL"};
        int v;
        if (!lookup(kPT, *t, v)) throw std::runtime_error("Invalid parameter type for " + p.name);
        p.type = ParamType(v);
      }
      p.typed = typed_param(p);
      u.parameters.push_back(std::move(p));
    }
  }
  u.model_uri = str_of(field2(j, "modelUri", "model_uri"));
  u.service_account_name = str_of(field2(j, "serviceAccountName", "service_account_name"));
  u.env_secret_ref_name = str_of(field2(j, "envSecretRefName", "env_secret_ref_name"));
  if (const Json* d = j.find("device"); d && d->is_number()) u.device = int(d->as_number());
  if (auto it = images.find(u.name); it != images.end()) {
    u.image = it->second;
    auto pos = u.image.rfind(':');
    if (pos != std::string::npos) {
      u.image_name = u.image.substr(0, pos);
      u.image_version = u.image.substr(pos + 1);
    } else {
      u.image_name = u.image;
    }
  }
  if (const Json* cs = j.find("children"); cs && cs->is_array()) {
    for (const auto& c : cs->items()) {
      u.children.emplace_back();
      parse_unit(c, u.children.back(), images);
    }
  }
}

void str_map(const Json* j, std::map<std::string, std::string>& out) {
  if (!j || !j->is_object()) return;
  for (const auto& kv : j->members()) out[kv.first] = str_of(&kv.second);
}

}  // namespace

const char* unit_type_name(UnitType t) { return kTypeNames[int(t)]; }
const char* unit_impl_name(UnitImpl i) { return kImplNames[int(i)]; }
const char* method_name(Method m) { return kMethodNames[int(m)]; }
bool parse_unit_type(const std::string& s, UnitType& out) { int v; if (!lookup(kTypeNames, Json(s), v)) return false; out = UnitType(v); return true; }
bool parse_unit_impl(const std::string& s, UnitImpl& out) { int v; if (!lookup(kImplNames, Json(s), v)) return false; out = UnitImpl(v); return true; }
bool parse_method(const std::string& s, Method& out) { int v; if (!lookup(kMethodNames, Json(s), v)) return false; out = Method(v); return true; }

const Parameter* UnitSpec::param(const std::string& n) const {
  for (const auto& p : parameters)
    if (p.name == n) return &p;
  return nullptr;
}

PredictorSpecC parse_predictor_spec(const Json& j_in, const std::string& predictor) {
  const Json* j = &j_in;
  // Full SeldonDeployment?  spec.predictors[...]
  if (const Json* spec = j_in.find("spec"); spec && spec->is_object()) {
    const Json* preds = spec->find("predictors");
    if (!preds || !preds->is_array() || preds->items().empty())
      throw std::runtime_error("SeldonDeployment has no predictors");
    j = &preds->items()[0];
    if (!predictor.empty()) {
      bool found = false;
      for (const auto& p : preds->items())
        if (str_of(p.find("name")) == predictor) { j = &p; found = true; break; }
      if (!found) throw std::runtime_error("predictor " + predictor + " not found");
    }
  }
  if (!j->is_object()) throw std::runtime_error("predictor spec must be an object");
  PredictorSpecC ps;
  ps.raw = *j;
  ps.name = str_of(j->find("name"));
  if (const Json* r = j->find("replicas"); r && r->is_number()) ps.replicas = int(r->as_number());
  if (const Json* t = j->find("traffic"); t && t->is_number()) ps.traffic = int(t->as_number());
  str_map(j->find("annotations"), ps.annotations);
  str_map(j->find("labels"), ps.labels);
  if (const Json* cs = field2(*j, "componentSpecs", "component_specs"); cs && cs->is_array()) {
    for (const auto& podspec : cs->items()) {
      const Json* spec = podspec.find("spec");
      if (!spec) continue;
      const Json* containers = spec->find("containers");
      if (!containers || !containers->is_array()) continue;
      for (const auto& c : containers->items())
        ps.container_images[str_of(c.find("name"))] = str_of(c.find("image"));
    }
  }
  const Json* g = j->find("graph");
  if (!g) throw std::runtime_error("predictor spec has no graph");
  parse_unit(*g, ps.graph, ps.container_images);
  return ps;
}

PredictorSpecC default_predictor_spec() {
  Json j = parse_json(
      R"({"name":"basic-predictor","componentSpecs":[{}],)"
      R"("graph":{"name":"basic-pu","type":"MODEL","implementation":"SIMPLE_MODEL"}})");
  return parse_predictor_spec(j);
}

}  // namespace sca
