"""seldon_core.flask_utils -> seldon_core_amd.serving.errors (the exception
and its JSON reply; the native front end replaces the Flask request helpers)."""
from seldon_core_amd.serving.errors import SeldonMicroserviceException  # noqa: F401
