"""seldon_core.seldon_client -> seldon_core_amd.client."""
from seldon_core_amd.client import (SeldonCallCredentials, SeldonChannelCredentials, SeldonClient,  # noqa: F401
                                    SeldonClientCombine, SeldonClientException, SeldonClientFeedback,
                                    SeldonClientPrediction)
