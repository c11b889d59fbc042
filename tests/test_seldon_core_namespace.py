"""The reference's ``seldon_core`` Python namespace (python/seldon_core/*.py)
resolves to this package: user code keeps its imports.  Name lists are the
public functions / classes of the reference modules covered here; the
proto-side ``utils`` helpers are checked for behaviour, not only presence."""
import base64
import os

import numpy as np
import pytest

import seldon_core_amd as sca

REFERENCE_NAMES = {
    "utils": "json_to_seldon_message json_to_feedback json_to_seldon_messages seldon_message_to_json "
             "seldon_messages_to_json feedback_to_json get_data_from_proto grpc_datadef_to_array get_meta_from_proto "
             "array_to_rest_datadef array_to_grpc_datadef array_to_list_value construct_response_json "
             "construct_response extract_request_parts_json extract_request_parts extract_feedback_request_parts",
    "metrics": "create_counter create_gauge create_timer validate_metrics",
    "user_model": "SeldonNotImplementedError SeldonComponent client_custom_tags client_class_names client_predict "
                  "client_transform_input client_transform_output client_custom_metrics client_feature_names "
                  "client_send_feedback client_route client_aggregate",
    "flask_utils": "SeldonMicroserviceException",
    "seldon_client": "SeldonClient SeldonClientPrediction SeldonClientFeedback SeldonClientCombine "
                     "SeldonChannelCredentials SeldonCallCredentials SeldonClientException",
    "storage": "Storage",
    "persistence": "restore persist PersistenceThread",
    "serving_test_gen": "create_seldon_api_testing_file",
    "microservice": "main",
    "wrapper": "get_rest_microservice",
}


@pytest.mark.parametrize("module", sorted(REFERENCE_NAMES))
def test_reference_module_names_resolve(module):
    import importlib

    mod = importlib.import_module(f"seldon_core.{module}")
    missing = [n for n in REFERENCE_NAMES[module].split() if not hasattr(mod, n)]
    assert not missing, missing


def test_reference_names_are_the_reference_modules_public_api():
    """Where the reference tree is present, its modules define (at least) the
    names listed above -- the list is not invented."""
    import re

    root = "/root/reference/python/seldon_core"
    if not os.path.isdir(root):
        pytest.skip("reference tree absent")
    for module in ("utils", "metrics", "user_model", "storage"):
        src = open(os.path.join(root, module + ".py")).read()
        defined = set(re.findall(r"^(?:def|class) (\w+)", src, re.M))
        listed = set(REFERENCE_NAMES[module].split())
        assert listed <= defined | {"SeldonNotImplementedError"}, listed - defined


def test_proto_helpers_round_trip_every_payload_kind():
    from seldon_core.proto import prediction_pb2
    from seldon_core.utils import (array_to_grpc_datadef, get_data_from_proto, get_meta_from_proto,
                                   grpc_datadef_to_array, json_to_seldon_message, seldon_message_to_json)

    X = np.arange(6.0).reshape(2, 3)
    for kind in ("tensor", "ndarray", "tftensor"):
        dd = array_to_grpc_datadef(kind, X, ["a", "b", "c"])
        assert isinstance(dd, prediction_pb2.DefaultData) and dd.WhichOneof("data_oneof") == kind
        np.testing.assert_array_equal(grpc_datadef_to_array(dd), X)
        msg = prediction_pb2.SeldonMessage(data=dd)
        np.testing.assert_array_equal(get_data_from_proto(msg), X)
        assert seldon_message_to_json(msg)["data"]["names"] == ["a", "b", "c"]
    m = json_to_seldon_message({"binData": base64.b64encode(b"\x00\x01").decode(), "meta": {"puid": "p1"}})
    assert get_data_from_proto(m) == b"\x00\x01" and get_meta_from_proto(m)["puid"] == "p1"
    assert get_data_from_proto(json_to_seldon_message({"strData": "hi"})) == "hi"
    assert get_data_from_proto(json_to_seldon_message({"jsonData": {"k": [1, 2]}})) == {"k": [1.0, 2.0]}
    from seldon_core.flask_utils import SeldonMicroserviceException

    with pytest.raises(SeldonMicroserviceException):
        json_to_seldon_message({"data": {"bogus": 1}})


def test_construct_response_and_feedback_parts():
    from seldon_core.utils import (construct_response, extract_feedback_request_parts, extract_request_parts,
                                   json_to_feedback, json_to_seldon_message, seldon_message_to_json)

    class Model:
        class_names = ["p", "q"]

        def tags(self):
            return {"model": "m"}

    req = json_to_seldon_message({"data": {"names": ["a", "b"], "tensor": {"shape": [1, 2], "values": [1, 2]}}})
    features, meta, datadef, kind = extract_request_parts(req)
    np.testing.assert_array_equal(features, [[1.0, 2.0]])
    assert kind == "data" and datadef.WhichOneof("data_oneof") == "tensor"
    out = seldon_message_to_json(construct_response(Model(), False, req, np.array([[0.25, 0.75]])))
    assert out["data"]["names"] == ["p", "q"]
    assert out["data"]["tensor"] == {"shape": [1, 2], "values": [0.25, 0.75]}  # the request's data type
    assert out["meta"]["tags"] == {"model": "m"}
    fb = json_to_feedback({"request": {"data": {"ndarray": [[1, 2]]}}, "truth": {"data": {"ndarray": [[1]]}},
                           "reward": 0.5})
    _, x, truth, reward = extract_feedback_request_parts(fb)
    np.testing.assert_array_equal(x, [[1.0, 2.0]])
    np.testing.assert_array_equal(truth, [[1.0]])
    assert reward == 0.5


def test_component_written_against_seldon_core_serves_and_keeps_its_error_contract():
    from seldon_core.flask_utils import SeldonMicroserviceException
    from seldon_core.metrics import create_counter
    from seldon_core.user_model import SeldonComponent

    class Doubler(SeldonComponent):
        def predict(self, X, names, meta=None):
            if np.asarray(X).min() < 0:
                raise SeldonMicroserviceException("negative input", status_code=422, reason="NEGATIVE")
            return np.asarray(X) * 2

        def metrics(self):
            return [create_counter("calls", 1)]

    spec = {"name": "p", "graph": {"name": "m", "type": "MODEL"}, "componentSpecs": [{"spec": {"containers": []}}]}
    dep = sca.Deployment(spec, device=-1, components={"m": Doubler()})
    try:
        out = dep.predict({"data": {"ndarray": [[1.0, 2.0]]}})
        assert out["data"]["ndarray"] == [[2.0, 4.0]]
        assert out["meta"]["metrics"][0]["key"] == "calls"
        with pytest.raises(Exception) as ei:
            dep.predict({"data": {"ndarray": [[-1.0, 2.0]]}})
        assert "422" in str(ei.value) or "NEGATIVE" in str(ei.value) or "negative input" in str(ei.value)
    finally:
        dep.close()


def test_wrapper_app_test_client_in_the_reference_call_shapes(tmp_path):
    """seldon_core.wrapper.get_rest_microservice(user_object).test_client():
    the reference's Flask-client call shapes against the native server."""
    import json

    from seldon_core.flask_utils import SeldonMicroserviceException
    from seldon_core.wrapper import get_rest_microservice

    class Echo:
        def __init__(self):
            self.rewards = []

        def predict(self, X, names):
            if isinstance(X, (bytes, bytearray)) or getattr(X, "dtype", None) is not None and X.dtype.kind == "S":
                return np.array([[len(bytes(np.asarray(X).tobytes()))]], dtype=float)
            X = np.asarray(X, dtype=float)
            if X.size and X.min() < 0:
                raise SeldonMicroserviceException("negative", status_code=402, reason="NEG")
            return X * 2

        def send_feedback(self, features, feature_names, reward, truth, routing=None):
            self.rewards.append(reward)

    comp = Echo()
    app = get_rest_microservice(comp)
    try:
        c = app.test_client()
        rv = c.get('/predict?json={"data":{"names":["a","b"],"ndarray":[[1,2]]}}')
        assert rv.status_code == 200 and rv.get_json()["data"]["ndarray"] == [[2.0, 4.0]]
        rv = c.post("/predict", data={"json": '{"data":{"ndarray":[[3,4]]}}'})
        assert rv.get_json()["data"]["ndarray"] == [[6.0, 8.0]]
        rv = c.post("/predict", data={"data": '{"names":["a","b"],"ndarray":[[1,2]]}'},
                    content_type="multipart/form-data")
        assert rv.status_code == 200 and rv.get_json()["data"]["ndarray"] == [[2.0, 4.0]]
        f = tmp_path / "test.txt"
        f.write_bytes(b"hello world")
        rv = c.post("/predict", data={"meta": '{"puid":"1234"}', "binData": (str(f), "test.txt")},
                    content_type="multipart/form-data")
        assert rv.status_code == 200, rv.data
        rv = c.get('/send-feedback?json={"request":{"data":{"ndarray":[]}},"reward":1.0}')
        assert rv.status_code == 200 and comp.rewards == [1.0]
        rv = c.get('/predict?json={"data":{"ndarray":[[-1,2]]}}')
        assert rv.status_code == 402 and json.loads(rv.data)["status"]["reason"] == "NEG"
    finally:
        app.close()
