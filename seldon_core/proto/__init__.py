"""seldon_core.proto -> seldon_core_amd.proto (wire-compatible prediction.proto)."""
from seldon_core_amd.proto import prediction_pb2  # noqa: F401
