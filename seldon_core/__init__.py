"""The reference's ``seldon_core`` Python namespace, answered by this package.

Code written against seldon-core's Python API keeps its imports::

    from seldon_core.seldon_client import SeldonClient
    from seldon_core.user_model import SeldonComponent
    from seldon_core.flask_utils import SeldonMicroserviceException
    from seldon_core.utils import json_to_seldon_message, get_data_from_proto
    from seldon_core.metrics import create_counter
    from seldon_core.proto import prediction_pb2

Every name here is the ``seldon_core_amd`` implementation (module docstrings
say which); nothing is re-implemented in this namespace.  Component classes
need none of it: they are duck-typed, as in the reference.
"""
from seldon_core_amd import __version__  # noqa: F401
