"""seldon_core_amd -- an MI355X-native inference-graph serving engine with the
capabilities of Seldon Core 0.5 (SeldonDeployment graphs, prediction.proto
REST/gRPC API, routers/combiners/transformers, feedback, metrics), executed
in-process by a native C++ graph executor with hand-written gfx950 kernels.
"""
from ._native import available as native_available, gpu_count, native
from .serving import (Deployment, EngineError, SeldonComponent, SeldonMicroserviceException,
                      SeldonNotImplementedError)
from .utils.storage import Storage


def __getattr__(name):  # the client pulls in protobuf / grpc: import it on first use
    if name == "_C":  # `from seldon_core_amd import _C`: through the loader, torch's HIP runtime first
        return native()
    if name in ("SeldonClient", "SeldonChannelCredentials", "SeldonCallCredentials"):
        from . import client

        return getattr(client, name)
    raise AttributeError(name)

__version__ = "0.1.0"

__all__ = ["Deployment", "EngineError", "SeldonComponent", "SeldonMicroserviceException",
           "SeldonNotImplementedError", "Storage", "native", "native_available", "gpu_count", "__version__"]
