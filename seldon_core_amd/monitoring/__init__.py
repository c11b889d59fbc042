"""Monitoring assets: Grafana dashboards and Prometheus rules for /prometheus."""
