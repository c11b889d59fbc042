#include "metrics.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "json.h"

namespace sca {

namespace {
inline double bits_to_d(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
inline uint64_t d_to_bits(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

void atomic_add_double(std::atomic<uint64_t>& a, double v) {
  uint64_t cur = a.load(std::memory_order_relaxed);
  while (!a.compare_exchange_weak(cur, d_to_bits(bits_to_d(cur) + v), std::memory_order_relaxed)) {}
}
void atomic_max_double(std::atomic<uint64_t>& a, double v) {
  uint64_t cur = a.load(std::memory_order_relaxed);
  while (bits_to_d(cur) < v && !a.compare_exchange_weak(cur, d_to_bits(v), std::memory_order_relaxed)) {}
}

constexpr double kBase = 1e-6;
const double kGrowth = std::pow(2.0, 1.0 / 8.0);

inline int bucket_of(double s) {
  if (!(s > kBase)) return 0;
  int b = int(8.0 * std::log2(s / kBase)) + 1;  // 2^(1/8) growth
  return std::min(b, Histogram::kBuckets - 1);
}
inline double bucket_upper(int b) { return kBase * std::pow(kGrowth, b); }

const double kLe[] = {0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0};
const double kQ[] = {0.5, 0.75, 0.95, 0.98, 0.99};

std::string sanitize(const std::string& n) {
  std::string o = n;
  for (auto& c : o)
    if (!(isalnum((unsigned char)c) || c == '_' || c == ':')) c = '_';
  if (!o.empty() && isdigit((unsigned char)o[0])) o = "_" + o;
  return o;
}
}  // namespace

namespace {
int stripe_of_this_thread() {
  static std::atomic<int> next{0};
  thread_local const int idx = next.fetch_add(1, std::memory_order_relaxed) % Histogram::kStripes;
  return idx;
}
}  // namespace

void Histogram::observe(double s) {
  Stripe& st = stripes_[stripe_of_this_thread()];
  st.buckets[bucket_of(s)].fetch_add(1, std::memory_order_relaxed);
  st.count.fetch_add(1, std::memory_order_relaxed);
  atomic_add_double(st.sum_bits, s);
  atomic_max_double(st.max_bits, s);
}

uint64_t Histogram::count() const {
  uint64_t n = 0;
  for (const auto& st : stripes_) n += st.count.load(std::memory_order_relaxed);
  return n;
}

double Histogram::sum() const {
  double v = 0.0;
  for (const auto& st : stripes_) v += bits_to_d(st.sum_bits.load(std::memory_order_relaxed));
  return v;
}

double Histogram::max() const {
  double v = 0.0;
  for (const auto& st : stripes_) v = std::max(v, bits_to_d(st.max_bits.load(std::memory_order_relaxed)));
  return v;
}

uint64_t Histogram::bucket_total(int b) const {
  uint64_t n = 0;
  for (const auto& st : stripes_) n += st.buckets[b].load(std::memory_order_relaxed);
  return n;
}

double Histogram::quantile(double q) const {
  uint64_t n = count();
  if (!n) return 0.0;
  uint64_t target = uint64_t(std::ceil(q * double(n)));
  if (target == 0) target = 1;
  uint64_t acc = 0;
  for (int b = 0; b < kBuckets; ++b) {
    acc += bucket_total(b);
    if (acc >= target) return std::min(bucket_upper(b), max());
  }
  return max();
}

uint64_t Histogram::count_le(double s) const {
  uint64_t acc = 0;
  for (int b = 0; b < kBuckets; ++b) {
    if (bucket_upper(b) > s * (1 + 1e-9)) break;
    acc += bucket_total(b);
  }
  return acc;
}

void Histogram::copy_from(const Histogram& o) {
  for (int i = 0; i < kStripes; ++i) {
    Stripe& d = stripes_[i];
    const Stripe& src = o.stripes_[i];
    for (int b = 0; b < kBuckets; ++b) d.buckets[b].store(src.buckets[b].load(std::memory_order_relaxed));
    d.count.store(src.count.load(std::memory_order_relaxed));
    d.sum_bits.store(src.sum_bits.load(std::memory_order_relaxed));
    d.max_bits.store(src.max_bits.load(std::memory_order_relaxed));
  }
}

void Histogram::reset() {
  for (auto& st : stripes_) {
    for (auto& b : st.buckets) b.store(0);
    st.count.store(0);
    st.sum_bits.store(0);
    st.max_bits.store(0);
  }
}

void Series::inc(double v) { atomic_add_double(value_bits, v); }
void Series::set(double v) { value_bits.store(d_to_bits(v), std::memory_order_relaxed); }
double Series::value() const { return bits_to_d(value_bits.load(std::memory_order_relaxed)); }

std::string render_labels(Labels labels) {
  std::sort(labels.begin(), labels.end());
  std::string s;
  for (const auto& kv : labels) {
    s += sanitize(kv.first);
    s += "=\"";
    for (char c : kv.second) {
      if (c == '"' || c == '\\') s.push_back('\\');
      if (c == '\n') { s += "\\n"; continue; }
      s.push_back(c);
    }
    s += "\",";
  }
  return s;
}

Series* MetricsRegistry::get(Series::Kind k, const std::string& family, Labels labels, bool q) {
  std::string l = render_labels(std::move(labels));
  std::string key = family + "{" + l;
  std::lock_guard<std::mutex> g(mu_);
  auto it = series_.find(key);
  if (it != series_.end()) return it->second.get();
  auto s = std::make_unique<Series>();
  s->kind = k;
  s->family = family;
  s->labels = std::move(l);
  s->quantiles = q;
  Series* raw = s.get();
  series_.emplace(std::move(key), std::move(s));
  return raw;
}

Series* MetricsRegistry::counter(const std::string& name, Labels labels) {
  return get(Series::Kind::Counter, sanitize(name) + "_total", std::move(labels), false);
}
Series* MetricsRegistry::gauge(const std::string& name, Labels labels) {
  return get(Series::Kind::Gauge, sanitize(name), std::move(labels), false);
}
Series* MetricsRegistry::timer(const std::string& name, Labels labels, bool quantiles) {
  return get(Series::Kind::Timer, sanitize(name) + "_seconds", std::move(labels), quantiles);
}

void MetricsRegistry::clear() {
  std::lock_guard<std::mutex> g(mu_);
  series_.clear();
}

std::string MetricsRegistry::render() const {
  std::lock_guard<std::mutex> g(mu_);
  std::string out;
  std::string last_family;
  // series_ is ordered by key (= family + labels) so families are contiguous.
  for (const auto& kv : series_) {
    const Series& s = *kv.second;
    if (s.family != last_family) {
      last_family = s.family;
      out += "# HELP " + s.family + " \n# TYPE " + s.family + " ";
      out += s.kind == Series::Kind::Counter ? "counter\n" : s.kind == Series::Kind::Gauge ? "gauge\n" : "histogram\n";
    }
    if (s.kind != Series::Kind::Timer) {
      out += s.family + "{" + s.labels + "} ";
      append_number(out, s.value());
      out.push_back('\n');
      continue;
    }
    const Histogram& h = s.hist;
    if (s.quantiles) {
      for (double q : kQ) {
        out += s.family + "{" + s.labels + "quantile=\"";
        append_number(out, q);
        out += "\",} ";
        append_number(out, h.quantile(q));
        out.push_back('\n');
      }
      for (double le : kLe) {
        out += s.family + "_bucket{" + s.labels + "le=\"";
        append_number(out, le);
        out += "\",} ";
        append_number(out, double(h.count_le(le)));
        out.push_back('\n');
      }
      out += s.family + "_bucket{" + s.labels + "le=\"+Inf\",} ";
      append_number(out, double(h.count()));
      out.push_back('\n');
    }
    out += s.family + "_count{" + s.labels + "} ";
    append_number(out, double(h.count()));
    out += "\n" + s.family + "_sum{" + s.labels + "} ";
    append_number(out, h.sum());
    out += "\n" + s.family + "_max{" + s.labels + "} ";
    append_number(out, h.max());
    out.push_back('\n');
  }
  return out;
}

}  // namespace sca
