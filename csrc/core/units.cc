// Built-in predictive units (engine/src/main/java/io/seldon/engine/predictors/
// SimpleModelUnit.java:37-63, SimpleRouterUnit.java:30-32,
// RandomABTestUnit.java:31-59, AverageCombinerUnit.java:35-79).
#include <mutex>

#include "engine.h"

namespace sca {
namespace {

const uint32_t kTI = method_bit(Method::TRANSFORM_INPUT);
const uint32_t kRO = method_bit(Method::ROUTE);
const uint32_t kAG = method_bit(Method::AGGREGATE);

MsgPtr branch_message(int branch) {
  auto m = std::make_shared<SeldonMessage>();
  m->payload = Payload::Data;
  m->data.kind = DataKind::Tensor;
  m->data.shape = {1, 1};
  m->data.values = {double(branch)};
  return m;
}

class SimpleModelUnit : public Unit {
 public:
  uint32_t builtin_methods() const override { return kTI; }
  std::string kind() const override { return "SIMPLE_MODEL"; }
  void transform_input(const CallCtx&, MsgPtr in, Done k) override {
    auto m = std::make_shared<SeldonMessage>();
    m->has_status = true;
    m->has_meta = true;
    m->meta.metrics = {Metric{"mymetric_counter", MetricType::COUNTER, 1.f, {}},
                       Metric{"mymetric_gauge", MetricType::GAUGE, 100.f, {}},
                       Metric{"mymetric_timer", MetricType::TIMER, 22.1f, {}}};
    if (in->payload == Payload::BinData) {
      m->payload = Payload::BinData;
      m->bin_data = in->bin_data;
    } else if (in->payload == Payload::StrData) {
      m->payload = Payload::StrData;
      m->str_data = in->str_data;
    } else {
      m->payload = Payload::Data;
      m->data.names = {"class0", "class1", "class2"};
      m->data.kind = DataKind::Tensor;
      m->data.shape = {1, 3};
      m->data.values = {0.1, 0.9, 0.5};
    }
    k(Outcome::ok(std::move(m)));
  }
};

class SimpleRouterUnit : public Unit {
 public:
  uint32_t builtin_methods() const override { return kRO; }
  std::string kind() const override { return "SIMPLE_ROUTER"; }
  void route(const CallCtx&, MsgPtr, Done k) override { k(Outcome::ok(branch_message(0))); }
};

class RandomABTestUnit : public Unit {
 public:
  explicit RandomABTestUnit(const UnitSpec& s) : rng_(1337) {
    if (const Parameter* p = s.param("ratioA")) {
      has_ratio_ = true;
      ratio_a_ = float(p->typed.is_number() ? p->typed.as_number() : atof(p->value.c_str()));
    }
  }
  uint32_t builtin_methods() const override { return kRO; }
  std::string kind() const override { return "RANDOM_ABTEST"; }
  void route(const CallCtx& c, MsgPtr, Done k) override {
    if (!has_ratio_) {
      k(Outcome::fail(make_error(ApiError::INVALID_ABTEST, "Parameter 'ratioA' is missing.")));
      return;
    }
    float cmp;
    {
      std::lock_guard<std::mutex> g(mu_);
      cmp = rng_.next_float();
    }
    size_t nchildren = c.node->children.size();
    if (nchildren != 2) {
      k(Outcome::fail(make_error(ApiError::INVALID_ABTEST, "AB test has " + std::to_string(nchildren) + " children ")));
      return;
    }
    k(Outcome::ok(branch_message(cmp <= ratio_a_ ? 0 : 1)));
  }
  std::string snapshot() const override {
    std::lock_guard<std::mutex> g(mu_);
    return std::to_string(rng_.state());
  }
  void restore(const std::string& s) override {
    std::lock_guard<std::mutex> g(mu_);
    rng_.set_state(std::stoull(s));
  }

 private:
  mutable std::mutex mu_;
  JavaRandom rng_;
  bool has_ratio_ = false;
  float ratio_a_ = 0.5f;
};

// Shape as the reference reads it (PredictorUtils.getShape): tensor shape, or
// [rows, cols-of-first-row] for ndarray.
bool combiner_shape(const DefaultData& d, std::vector<int64_t>& shape) {
  if (d.kind == DataKind::Tensor) { shape = d.shape; return true; }
  if (d.kind == DataKind::NdArray) {
    std::vector<double> tmp;
    return d.dense(shape, tmp, nullptr) || (!shape.empty());
  }
  if (d.kind == DataKind::TfTensor) { shape = d.tftensor.dims; return true; }
  return false;
}

class AverageCombinerUnit : public Unit {
 public:
  uint32_t builtin_methods() const override { return kAG; }
  std::string kind() const override { return "AVERAGE_COMBINER"; }
  void aggregate(const CallCtx&, std::vector<MsgPtr> outs, Done k) override {
    if (outs.empty()) {
      k(Outcome::fail(make_error(ApiError::INVALID_COMBINER_RESPONSE, "Combiner received no inputs")));
      return;
    }
    std::vector<int64_t> shape;
    if (outs[0]->payload != Payload::Data || !combiner_shape(outs[0]->data, shape)) {
      k(Outcome::fail(make_error(ApiError::INVALID_COMBINER_RESPONSE, "Combiner cannot extract data shape")));
      return;
    }
    if (shape.size() != 2) {
      k(Outcome::fail(make_error(ApiError::INVALID_COMBINER_RESPONSE, "Combiner received data that is not 2 dimensional")));
      return;
    }
    std::vector<double> sum(size_t(shape[0] * shape[1]), 0.0);
    std::vector<int64_t> s;
    std::vector<double> v;
    for (const auto& o : outs) {
      std::string err;
      if (o->payload != Payload::Data || !o->data.dense(s, v, &err)) {
        k(Outcome::fail(make_error(ApiError::INVALID_COMBINER_RESPONSE, "Combiner cannot extract data shape")));
        return;
      }
      if (s.size() != 2) {
        k(Outcome::fail(make_error(ApiError::INVALID_COMBINER_RESPONSE, "Combiner received data that is not 2 dimensional")));
        return;
      }
      if (s[0] != shape[0]) {
        k(Outcome::fail(make_error(ApiError::INVALID_COMBINER_RESPONSE,
                                   "Expected batch length " + std::to_string(shape[0]) + " but found " + std::to_string(s[0]))));
        return;
      }
      if (s[1] != shape[1]) {
        k(Outcome::fail(make_error(ApiError::INVALID_COMBINER_RESPONSE,
                                   "Expected batch length " + std::to_string(shape[1]) + " but found " + std::to_string(s[1]))));
        return;
      }
      for (size_t i = 0; i < sum.size(); ++i) sum[i] += v[i];
    }
    const double inv = 1.0 / double(outs.size());
    for (auto& x : sum) x *= inv;
    auto m = std::make_shared<SeldonMessage>();
    m->payload = Payload::Data;
    m->data.names = outs[0]->data.names;
    m->data.set_dense(outs[0]->data.kind, shape, std::move(sum));
    m->has_meta = outs[0]->has_meta;
    m->meta = outs[0]->meta;
    m->has_status = outs[0]->has_status;
    m->status = outs[0]->status;
    k(Outcome::ok(std::move(m)));
  }
};

}  // namespace

UnitPtr make_builtin_unit(UnitImpl impl, const UnitSpec& spec) {
  switch (impl) {
    case UnitImpl::SIMPLE_MODEL: return std::make_shared<SimpleModelUnit>();
    case UnitImpl::SIMPLE_ROUTER: return std::make_shared<SimpleRouterUnit>();
    case UnitImpl::RANDOM_ABTEST: return std::make_shared<RandomABTestUnit>(spec);
    case UnitImpl::AVERAGE_COMBINER: return std::make_shared<AverageCombinerUnit>();
    default: return nullptr;
  }
}

}  // namespace sca
