"""Serving layer: component API, codecs, dispatch, deployments."""
from .deployment import Deployment, ServerHandle
from .errors import EngineError, SeldonMicroserviceException, SeldonNotImplementedError
from .user_model import SeldonComponent

__all__ = ["Deployment", "ServerHandle", "EngineError", "SeldonMicroserviceException",
           "SeldonNotImplementedError", "SeldonComponent"]
