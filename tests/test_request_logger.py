"""Request-logger sink (reference seldon-request-logger/app/app.py) fed by the
engine's CloudEvents message logger."""
import io
import json
import time

import seldon_core_amd as sca
from seldon_core_amd.request_logger import flatten_pair, serve
from seldon_core_amd.serving.config import EngineConfig


def test_flatten_pair_rows():
    content = {"request": {"data": {"names": ["a", "b"], "ndarray": [[1, 2], [3, 4]]}, "date": "d1"},
               "response": {"data": {"names": ["p"], "tensor": {"shape": [2, 1], "values": [0.1, 0.9]}},
                            "meta": {"puid": "x"}, "date": "d2"},
               "sdepName": "dep"}
    docs = flatten_pair(content)
    assert len(docs) == 2
    assert docs[0]["request_elements"] == {"a": [1], "b": [2]}
    assert docs[1]["response_elements"] == {"p": [0.9]}
    assert docs[1]["request"]["dataType"] == "tabular"
    assert docs[1]["request"]["tabular"]["data"]["ndarray"] == [[3, 4]]
    assert docs[0]["response"]["tabular"]["meta"] == {"puid": "x"}
    assert docs[0]["sdepName"] == "dep"


def test_flatten_request_only_and_passthrough():
    docs = flatten_pair({"request": {"data": {"ndarray": [[1.0, 2.0]]}}})
    assert docs[0]["request_elements"] == {"t:0": [1.0], "t:1": [2.0]}
    assert flatten_pair({"other": 1}) == [{"other": 1}]


def test_engine_to_logger_end_to_end():
    buf = io.StringIO()
    srv = serve("127.0.0.1", 0, out=buf)
    try:
        cfg = EngineConfig.resolve(env={"SELDON_LOG_MESSAGES_EXTERNALLY": "true", "DEPLOYMENT_NAME": "d",
                                        "SELDON_MESSAGE_LOGGING_SERVICE": f"http://127.0.0.1:{srv.server_port}"},
                                   annotations_file="/nonexistent")
        dep = sca.Deployment(None, device=-1, config=cfg)
        try:
            dep.predict({"data": {"names": ["x", "y"], "ndarray": [[1.0, 2.0]]}})
            dep.engine.flush_message_log()
        finally:
            dep.close()
        for _ in range(100):
            if buf.getvalue():
                break
            time.sleep(0.01)
        doc = json.loads(buf.getvalue().splitlines()[0])
        assert doc["request_elements"] == {"x": [1.0], "y": [2.0]}
        assert doc["response_elements"] == {"class0": [0.1], "class1": [0.9], "class2": [0.5]}
        assert doc["sdepName"] == "d"
    finally:
        srv.shutdown()
