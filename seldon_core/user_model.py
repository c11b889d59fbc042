"""seldon_core.user_model -> seldon_core_amd.serving.user_model."""
from seldon_core_amd.serving.errors import SeldonNotImplementedError  # noqa: F401
from seldon_core_amd.serving.user_model import (SeldonComponent, client_aggregate, client_class_names,  # noqa: F401
                                                client_custom_metrics, client_custom_tags, client_feature_names,
                                                client_predict, client_route, client_send_feedback,
                                                client_transform_input, client_transform_output)
