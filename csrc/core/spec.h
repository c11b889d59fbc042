// PredictorSpec / PredictiveUnit model (reference proto/seldon_deployment.proto:11-161,
// engine/.../predictors/EnginePredictor.java:58-158, PredictorBean.java:51-83,
// PredictiveUnitState.java:37-125).
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "json.h"

namespace sca {

enum class UnitType : int { UNKNOWN_TYPE = 0, ROUTER = 1, COMBINER = 2, MODEL = 3, TRANSFORMER = 4, OUTPUT_TRANSFORMER = 5 };
enum class UnitImpl : int {
  UNKNOWN_IMPLEMENTATION = 0, SIMPLE_MODEL = 1, SIMPLE_ROUTER = 2, RANDOM_ABTEST = 3,
  AVERAGE_COMBINER = 4, SKLEARN_SERVER = 5, XGBOOST_SERVER = 6, TENSORFLOW_SERVER = 7, MLFLOW_SERVER = 8
};
enum class Method : int { TRANSFORM_INPUT = 0, TRANSFORM_OUTPUT = 1, ROUTE = 2, AGGREGATE = 3, SEND_FEEDBACK = 4 };
enum class EndpointType : int { REST = 0, GRPC = 1 };
enum class ParamType : int { INT = 0, FLOAT = 1, DOUBLE = 2, STRING = 3, BOOL = 4 };

inline uint32_t method_bit(Method m) { return 1u << int(m); }

const char* unit_type_name(UnitType t);
const char* unit_impl_name(UnitImpl i);
const char* method_name(Method m);
bool parse_unit_type(const std::string& s, UnitType& out);
bool parse_unit_impl(const std::string& s, UnitImpl& out);
bool parse_method(const std::string& s, Method& out);

struct Parameter {
  std::string name;
  std::string value;
  ParamType type = ParamType::STRING;
  Json typed;  // value converted per type (PredictiveUnitParameter.fromParameter)
};

struct UnitSpec {
  std::string name;
  std::vector<UnitSpec> children;
  bool has_type = false;
  UnitType type = UnitType::UNKNOWN_TYPE;
  UnitImpl implementation = UnitImpl::UNKNOWN_IMPLEMENTATION;
  std::string implementation_name;  // raw string (allows engine-native extensions)
  std::vector<Method> methods;
  std::string service_host;
  int service_port = 0;
  EndpointType endpoint_type = EndpointType::REST;
  std::vector<Parameter> parameters;
  std::string model_uri;
  std::string service_account_name;
  std::string env_secret_ref_name;
  // Resolved from componentSpecs (PredictorBean.java:67-83).
  std::string image;          // full image string, "" when unknown
  std::string image_name;     // before ':'
  std::string image_version;  // after ':'
  // MI355X extension: placement (-1 = engine default).
  int device = -1;

  const Parameter* param(const std::string& n) const;
};

struct PredictorSpecC {
  std::string name;
  UnitSpec graph;
  int replicas = 1;
  int traffic = 0;
  std::map<std::string, std::string> annotations;
  std::map<std::string, std::string> labels;
  std::map<std::string, std::string> container_images;  // container name -> image
  Json raw;
};

// Accepts a bare PredictorSpec JSON or a full SeldonDeployment (first
// predictor, or the one named `predictor`).  Throws std::runtime_error.
PredictorSpecC parse_predictor_spec(const Json& j, const std::string& predictor = "");

// Default graph when no spec is supplied (EnginePredictor.java:122-141).
PredictorSpecC default_predictor_spec();

}  // namespace sca
