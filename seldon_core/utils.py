"""seldon_core.utils -> seldon_core_amd.serving.proto_utils (proto side) and
seldon_core_amd.serving.codec (JSON side)."""
from seldon_core_amd.serving.codec import (array_to_rest_datadef, construct_response_json,  # noqa: F401
                                           extract_request_parts_json)
from seldon_core_amd.serving.proto_utils import (array_to_grpc_datadef, array_to_list_value,  # noqa: F401
                                                 construct_response, extract_feedback_request_parts,
                                                 extract_request_parts, feedback_to_json, get_data_from_proto,
                                                 get_meta_from_proto, grpc_datadef_to_array, json_to_feedback,
                                                 json_to_seldon_message, json_to_seldon_messages,
                                                 seldon_message_to_json, seldon_messages_to_json)
