"""seldon_core.metrics -> seldon_core_amd.serving.metrics."""
from seldon_core_amd.serving.metrics import create_counter, create_gauge, create_timer, validate_metrics  # noqa: F401
