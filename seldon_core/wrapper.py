"""seldon_core.wrapper -> seldon_core_amd.microservice (the app is the native
internal-API server; ``test_client()`` and ``run()`` as on the Flask app)."""
from seldon_core_amd.microservice import MicroserviceApp, get_rest_microservice  # noqa: F401
