"""Grafana dashboards and Prometheus rules for the engine's /prometheus
endpoint (reference helm-charts/seldon-core-analytics/files/grafana/
configs/predictions-analytics-dashboard.json, outlier-detection-*.json and
monitoring/prometheus).

The dashboards are generated (``python -m seldon_core_amd.monitoring.dashboards
--out monitoring/``) rather than hand-edited exports, so every PromQL
expression is built from the metric names and labels the native registry
actually emits (csrc/core/metrics.cc; tests/test_monitoring.py scrapes a live
engine and checks each referenced series exists):

* ``prediction-analytics`` -- the reference dashboard's panels: global / per
  deployment request rate, success ratio, 4xx / 5xx, per-model request rate,
  feedback reward ratio, latency quantiles from the histogram buckets.
* ``gpu-serving`` -- MI355X micro-batcher series (``seldon_gpu_*``): batches /
  s, rows per batch, requests per batch, device busy fraction per slot,
  in-flight rows, per device and replica.
* ``outlier-detection`` -- the outlier detectors' custom gauges
  (``is_outlier``, scores, confusion counts, rolling F1 / precision / recall).
* ``multi-armed-bandit`` -- per-branch reward ratio and traffic under a router.
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Dict, List

DS = "prometheus"
SEL = 'deployment_name=~"$deployment",predictor_name=~"$predictor",model_name=~"$model_name"'


def _target(expr: str, legend: str = "", ref: str = "A") -> Dict:
    return {"expr": expr, "legendFormat": legend, "refId": ref, "intervalFactor": 1}


class _Board:
    def __init__(self, uid: str, title: str, tags: List[str]):
        self.d = {"uid": uid, "title": title, "tags": tags, "schemaVersion": 16, "version": 1, "editable": True,
                  "time": {"from": "now-15m", "to": "now"}, "refresh": "5s", "timezone": "browser",
                  "templating": {"list": []}, "panels": [], "annotations": {"list": []}}
        self._x = self._y = 0

    def var(self, name: str, query: str) -> "_Board":
        self.d["templating"]["list"].append({
            "name": name, "label": name, "type": "query", "datasource": DS, "refresh": 2, "includeAll": True,
            "multi": True, "allValue": ".*", "query": query, "current": {"text": "All", "value": "$__all"}})
        return self

    def _pos(self, w: int, h: int) -> Dict:
        if self._x + w > 24:
            self._x, self._y = 0, self._y + h
        p = {"x": self._x, "y": self._y, "w": w, "h": h}
        self._x += w
        return p

    def stat(self, title: str, expr: str, unit: str = "none", w: int = 6) -> "_Board":
        self.d["panels"].append({"id": len(self.d["panels"]) + 1, "type": "singlestat", "title": title,
                                 "datasource": DS, "format": unit, "gridPos": self._pos(w, 4),
                                 "targets": [_target(expr)], "valueName": "current", "sparkline": {"show": True}})
        return self

    def graph(self, title: str, targets: List[Dict], unit: str = "short", w: int = 12) -> "_Board":
        for i, t in enumerate(targets):
            t["refId"] = chr(ord("A") + i)
        self.d["panels"].append({"id": len(self.d["panels"]) + 1, "type": "graph", "title": title, "datasource": DS,
                                 "gridPos": self._pos(w, 8), "targets": targets, "lines": True, "linewidth": 1,
                                 "yaxes": [{"format": unit, "show": True}, {"format": "short", "show": False}],
                                 "legend": {"show": True, "values": False}})
        return self


def prediction_analytics() -> Dict:
    srv = "seldon_api_engine_server_requests_seconds"
    cli = "seldon_api_engine_client_requests_seconds"
    b = _Board("seldon-prediction-analytics", "Prediction Analytics", ["seldon", "serving"])
    b.var("deployment", f"label_values({srv}_count, deployment_name)")
    b.var("predictor", f'label_values({cli}_count{{deployment_name=~"$deployment"}}, predictor_name)')
    b.var("model_name", f'label_values({cli}_count{{deployment_name=~"$deployment"}}, model_name)')
    b.stat("Global Request Rate", f"round(sum(irate({srv}_count[1m])), 0.001)", "reqps")
    b.stat("Success", f'sum(rate({srv}_count{{status!~"5.*"}}[1m])) / sum(rate({srv}_count[1m]))', "percentunit")
    b.stat("4xxs", f'sum(irate({srv}_count{{status=~"4.*"}}[1m]))', "reqps")
    b.stat("5xxs", f'sum(irate({srv}_count{{status=~"5.*"}}[1m]))', "reqps")
    b.stat("Request Rate ($deployment)",
           f'round(sum(irate({srv}_count{{deployment_name=~"$deployment",uri=~".*predictions"}}[1m])), 0.001)', "reqps")
    b.stat("Success ($deployment)",
           f'sum(rate({srv}_count{{deployment_name=~"$deployment",status!~"5.*"}}[1m])) / '
           f'sum(rate({srv}_count{{deployment_name=~"$deployment"}}[1m]))', "percentunit")
    b.stat("p99 latency ($deployment)",
           f'max({srv}{{deployment_name=~"$deployment",uri=~".*predictions",quantile="0.99"}})', "s")
    b.stat("Feedback rate ($deployment)",
           f'sum(irate(seldon_api_model_feedback_total{{deployment_name=~"$deployment"}}[1m]))', "reqps")
    b.graph("Reqs/sec per model", [_target(
        f'sum(rate({cli}_count{{{SEL}}}[1m])) by (model_name,predictor_name,predictor_version,model_image,'
        f'model_version)', "{{model_name}} {{predictor_name}} {{model_version}}")], "reqps")
    b.graph("Model reward ratio", [_target(
        f'rate(seldon_api_model_feedback_reward_total{{{SEL}}}[1m]) / '
        f'rate(seldon_api_model_feedback_total{{{SEL}}}[1m])', "{{model_name}} {{predictor_name}}")], "percentunit")
    b.graph("Model latency", [
        _target(f'histogram_quantile({q}, sum(rate({cli}_bucket{{uri="/predict",{SEL}}}[20s])) by '
                f'(predictor_name,model_name,model_version,le))', f"p{int(q * 100)} {{{{model_name}}}}")
        for q in (0.5, 0.75, 0.9, 0.99)], "s")
    b.graph("Engine latency quantiles", [
        _target(f'max({srv}{{deployment_name=~"$deployment",uri=~".*predictions",quantile="{q}"}})', f"q{q}")
        for q in ("0.5", "0.95", "0.99")], "s")
    b.graph("Requests by status", [_target(
        f'sum(rate({srv}_count{{deployment_name=~"$deployment"}}[1m])) by (status,uri)', "{{status}} {{uri}}")],
        "reqps")
    return b.d


def gpu_serving() -> Dict:
    lab = f'{SEL},device=~"$device"'
    b = _Board("seldon-gpu-serving", "MI355X Serving (micro-batchers)", ["seldon", "gpu"])
    b.var("deployment", "label_values(seldon_gpu_batches_total, deployment_name)")
    b.var("predictor", 'label_values(seldon_gpu_batches_total{deployment_name=~"$deployment"}, predictor_name)')
    b.var("model_name", 'label_values(seldon_gpu_batches_total{deployment_name=~"$deployment"}, model_name)')
    b.var("device", "label_values(seldon_gpu_batches_total, device)")
    b.stat("GPU batches / s", f"sum(rate(seldon_gpu_batches_total{{{lab}}}[1m]))", "ops")
    b.stat("Rows / batch", f"sum(rate(seldon_gpu_rows_total{{{lab}}}[1m])) / "
                           f"sum(rate(seldon_gpu_batches_total{{{lab}}}[1m]))")
    b.stat("Device busy (per slot)", f"sum(rate(seldon_gpu_busy_seconds_total{{{lab}}}[1m])) / "
                                     f"sum(seldon_gpu_slots{{{lab}}})", "percentunit")
    b.stat("In-flight rows", f"sum(seldon_gpu_inflight_rows{{{lab}}})")
    b.graph("Batches / s by device", [_target(
        f"sum(rate(seldon_gpu_batches_total{{{lab}}}[1m])) by (model_name,device,replica)",
        "{{model_name}} gpu{{device}} r{{replica}}")], "ops")
    b.graph("Rows per batch", [_target(
        f"sum(rate(seldon_gpu_rows_total{{{lab}}}[1m])) by (model_name,device) / "
        f"sum(rate(seldon_gpu_batches_total{{{lab}}}[1m])) by (model_name,device)", "{{model_name}} gpu{{device}}"),
        _target(f"max(seldon_gpu_max_batch_rows{{{lab}}}) by (model_name)", "max {{model_name}}")])
    b.graph("Requests per batch", [_target(
        f"sum(rate(seldon_gpu_requests_total{{{lab}}}[1m])) by (model_name,device) / "
        f"sum(rate(seldon_gpu_batches_total{{{lab}}}[1m])) by (model_name,device)", "{{model_name}} gpu{{device}}")])
    b.graph("Device busy fraction per slot", [_target(
        f"sum(rate(seldon_gpu_busy_seconds_total{{{lab}}}[1m])) by (model_name,device) / "
        f"sum(seldon_gpu_slots{{{lab}}}) by (model_name,device)", "{{model_name}} gpu{{device}}")], "percentunit")
    b.graph("In-flight rows", [_target(f"sum(seldon_gpu_inflight_rows{{{lab}}}) by (model_name,device,replica)",
                                       "{{model_name}} gpu{{device}} r{{replica}}")])
    b.graph("Per-replica request share", [_target(
        f"sum(rate(seldon_gpu_requests_total{{{lab}}}[1m])) by (model_name,replica) / ignoring(replica) "
        f"group_left sum(rate(seldon_gpu_requests_total{{{lab}}}[1m])) by (model_name)",
        "{{model_name}} r{{replica}}")], "percentunit")
    return b.d


OUTLIER_GAUGES = ["observation", "is_outlier", "label", "nb_outliers_tot", "nb_labels_tot", "nb_outliers_roll",
                  "nb_labels_roll", "true_positive", "false_positive", "true_negative", "false_negative",
                  "accuracy_tot", "precision_tot", "recall_tot", "f1_tot", "f1_roll", "f2_roll", "accuracy_roll",
                  "precision_roll", "recall_roll"]


def outlier_detection(score_key: str = "outlier_score") -> Dict:
    b = _Board(f"seldon-outlier-{score_key}", f"Outlier Detection ({score_key})", ["seldon", "outliers"])
    b.var("model_name", "label_values(is_outlier, model_name)")
    m = '{model_name=~"$model_name"}'
    b.stat("Nb observations", f"max(observation{m})")
    b.stat("Nb Predicted Outliers", f"max(nb_outliers_tot{m})")
    b.stat("% Predicted Outliers", f"100 * max(nb_outliers_tot{m}) / max(observation{m})", "percent")
    b.stat("Nb Labeled Outliers", f"max(nb_labels_tot{m})")
    b.graph("Outlier Prediction", [_target(f"is_outlier{m}", "{{model_name}}")])
    b.graph("Outlier Score", [_target(f"{score_key}{m}", "{{model_name}}"),
                              _target(f"threshold{m}", "threshold")])
    b.graph("Outlier Labels", [_target(f"label{m}", "{{model_name}}")])
    b.graph("Rolling Number of Predicted and Labeled Outliers",
            [_target(f"nb_outliers_roll{m}", "predicted"), _target(f"nb_labels_roll{m}", "labeled")])
    for k, t in (("true_positive", "True Positive"), ("false_positive", "False Positive"),
                 ("true_negative", "True Negative"), ("false_negative", "False Negative"),
                 ("f1_tot", "F1 score"), ("accuracy_tot", "Accuracy"), ("precision_tot", "Precision"),
                 ("recall_tot", "Recall")):
        b.stat(t, f"max({k}{m})")
    b.graph("Rolling F1 and F2 Scores", [_target(f"f1_roll{m}", "F1"), _target(f"f2_roll{m}", "F2")])
    b.graph("Rolling Accuracy, Precision and Recall Scores",
            [_target(f"accuracy_roll{m}", "accuracy"), _target(f"precision_roll{m}", "precision"),
             _target(f"recall_roll{m}", "recall")])
    return b.d


def multi_armed_bandit() -> Dict:
    cli = "seldon_api_engine_client_requests_seconds"
    b = _Board("seldon-mab", "Multi-Armed Bandit", ["seldon", "routers"])
    b.var("deployment", f"label_values({cli}_count, deployment_name)")
    sel = 'deployment_name=~"$deployment"'
    b.graph("Reward ratio per branch", [_target(
        f"sum(rate(seldon_api_model_feedback_reward_total{{{sel}}}[1m])) by (model_name) / "
        f"sum(rate(seldon_api_model_feedback_total{{{sel}}}[1m])) by (model_name)", "{{model_name}}")],
        "percentunit", w=24)
    b.graph("Traffic per branch", [_target(
        f'sum(rate({cli}_count{{{sel},uri="/predict"}}[1m])) by (model_name)', "{{model_name}}")], "reqps")
    b.graph("Cumulative feedback per branch", [_target(
        f"sum(seldon_api_model_feedback_total{{{sel}}}) by (model_name)", "{{model_name}}")])
    return b.d


def prometheus_rules() -> str:
    srv = "seldon_api_engine_server_requests_seconds"
    rules = [
        ("SeldonHighErrorRate", f'sum(rate({srv}_count{{status=~"5.*"}}[5m])) by (deployment_name) / '
                                f"sum(rate({srv}_count[5m])) by (deployment_name) > 0.05", "2m",
         "More than 5% of requests to {{ $labels.deployment_name }} fail"),
        ("SeldonHighP99Latency", f'max({srv}{{quantile="0.99",uri=~".*predictions"}}) by (deployment_name) > 0.1',
         "5m", "p99 latency of {{ $labels.deployment_name }} above 100 ms"),
        ("SeldonGpuSaturated", "sum(rate(seldon_gpu_busy_seconds_total[5m])) by (device) / "
                               "sum(seldon_gpu_slots) by (device) > 0.9", "10m",
         "GPU {{ $labels.device }} micro-batchers busy > 90% per slot: add replicas / GPUs"),
        ("SeldonGpuBacklog", "sum(seldon_gpu_inflight_rows) by (device, model_name) > 8192", "2m",
         "{{ $labels.model_name }} on GPU {{ $labels.device }} has a growing row backlog"),
    ]
    lines = ["groups:", "- name: seldon-core-amd", "  rules:"]
    for name, expr, dur, summary in rules:
        lines += [f"  - alert: {name}", f"    expr: {json.dumps(expr)}", f"    for: {dur}",
                  "    labels:", "      severity: warning", "    annotations:", f"      summary: {json.dumps(summary)}"]
    return "\n".join(lines) + "\n"


def prometheus_scrape_config(targets: List[str]) -> str:
    t = ", ".join(json.dumps(x) for x in targets)
    return ("global:\n  scrape_interval: 5s\nrule_files:\n  - rules.yml\nscrape_configs:\n"
            f"- job_name: seldon-engine\n  metrics_path: /prometheus\n  static_configs:\n  - targets: [{t}]\n")


def all_dashboards() -> Dict[str, Dict]:
    return {"prediction-analytics": prediction_analytics(), "gpu-serving": gpu_serving(),
            "outlier-detection-md": outlier_detection("outlier_score"),
            "outlier-detection-vae": outlier_detection("mse"),
            "outlier-detection-if": outlier_detection("anomaly_score"),
            "multi-armed-bandit": multi_armed_bandit()}


def write(out_dir: str, targets: List[str]) -> List[str]:
    os.makedirs(os.path.join(out_dir, "grafana"), exist_ok=True)
    os.makedirs(os.path.join(out_dir, "prometheus"), exist_ok=True)
    paths = []
    for name, d in all_dashboards().items():
        p = os.path.join(out_dir, "grafana", f"{name}.json")
        with open(p, "w") as f:
            json.dump({"dashboard": d, "overwrite": True}, f, indent=1)
        paths.append(p)
    for fname, text in (("rules.yml", prometheus_rules()), ("prometheus.yml", prometheus_scrape_config(targets))):
        p = os.path.join(out_dir, "prometheus", fname)
        with open(p, "w") as f:
            f.write(text)
        paths.append(p)
    return paths


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="seldon-amd-dashboards")
    ap.add_argument("--out", default="monitoring")
    ap.add_argument("--target", action="append", default=None, help="engine host:port to scrape")
    a = ap.parse_args(argv)
    for p in write(a.out, a.target or ["127.0.0.1:8000"]):
        print(p)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
