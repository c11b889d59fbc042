// Prometheus metrics registry with the reference's metric names and tag keys
// (engine/src/main/resources/application.properties:4-10,
// engine/.../metrics/SeldonRestTemplateExchangeTagsProvider.java:38-154,
// engine/.../metrics/CustomMetricsManager.java:32-82,
// engine/.../predictors/PredictiveUnitBean.java:313-344).
//
// Updates are lock-free (atomics); only first creation of a series takes the
// registry mutex.  Rendering emits the Prometheus text format used by the
// reference's simpleclient (label lists end with ",}").
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace sca {

using Labels = std::vector<std::pair<std::string, std::string>>;

// Log-bucketed latency histogram.  Observations go to one of kStripes
// cache-line-aligned stripes chosen by the observing thread, so the front-end
// workers that time every request do not bounce one set of counters between
// cores; readers (scrapes) sum the stripes.
class Histogram {
 public:
  static constexpr int kBuckets = 240;  // 2^(1/8) spaced from 1us
  static constexpr int kStripes = 8;
  void observe(double seconds);
  double quantile(double q) const;
  uint64_t count() const;
  double sum() const;
  double max() const;
  uint64_t count_le(double seconds) const;
  void copy_from(const Histogram& o);  // snapshot (scrape-time export of a unit's own histogram)
  void reset();

 private:
  struct alignas(64) Stripe {
    std::atomic<uint64_t> buckets[kBuckets] = {};
    std::atomic<uint64_t> count{0};
    std::atomic<uint64_t> sum_bits{0};
    std::atomic<uint64_t> max_bits{0};
  };
  uint64_t bucket_total(int b) const;
  Stripe stripes_[kStripes];
};

struct Series {
  enum class Kind { Counter, Gauge, Timer };
  Kind kind;
  std::string family;   // rendered family name (with _total / _seconds suffix)
  std::string labels;   // rendered `k="v",...,`
  bool quantiles = false;
  std::atomic<uint64_t> value_bits{0};
  Histogram hist;

  void inc(double v = 1.0);
  void set(double v);
  double value() const;
  void observe_seconds(double s) { hist.observe(s); }
};

class MetricsRegistry {
 public:
  Series* counter(const std::string& name, Labels labels);
  Series* gauge(const std::string& name, Labels labels);
  // `quantiles` adds the 0.5/0.75/0.95/0.98/0.99 summary lines.
  Series* timer(const std::string& name, Labels labels, bool quantiles = false);
  std::string render() const;
  void clear();

 private:
  Series* get(Series::Kind k, const std::string& family, Labels labels, bool q);
  mutable std::mutex mu_;
  std::map<std::string, std::unique_ptr<Series>> series_;  // key: family + "{" + labels
};

std::string render_labels(Labels labels);

}  // namespace sca
