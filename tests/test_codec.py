"""Wire codecs: SeldonMessage JSON <-> native struct <-> protobuf.

Cases follow the reference's codec tests (python/tests/test_utils.py,
engine/src/test/java/io/seldon/engine/pb/TestJsonParse.java, TestPredictionProto.java).
"""
import base64
import json

import numpy as np
import pytest


def rt(C, obj):
    return json.loads(C.json_roundtrip(json.dumps(obj)))


def test_tensor_roundtrip(C):
    out = rt(C, {"data": {"names": ["a", "b"], "tensor": {"shape": [2, 2], "values": [1, 2.5, -3, 4e-9]}}})
    assert out["data"]["tensor"] == {"shape": [2, 2], "values": [1.0, 2.5, -3.0, 4e-9]}
    assert out["data"]["names"] == ["a", "b"]


def test_ndarray_mixed_roundtrip(C):
    nd = [[1, "a", None, True], [2.5, {"k": [1, 2]}, [], False]]
    out = rt(C, {"data": {"ndarray": nd}})
    assert out["data"]["ndarray"] == [[1.0, "a", None, True], [2.5, {"k": [1.0, 2.0]}, [], False]]


def test_meta_defaults_and_fields(C):
    msg = {"meta": {"puid": "abc", "tags": {"t": "v", "n": 1}, "routing": {"r": -1, "q": 2},
                    "requestPath": {"m": "img:1"},
                    "metrics": [{"key": "c", "type": "COUNTER", "value": 1}, {"key": "g", "type": "GAUGE", "value": 2.5,
                                                                            "tags": {"x": "y"}}]},
           "strData": "hello"}
    out = rt(C, msg)
    assert out["meta"]["puid"] == "abc"
    assert out["meta"]["routing"] == {"r": -1, "q": 2}
    assert out["meta"]["metrics"][1] == {"key": "g", "type": "GAUGE", "value": 2.5, "tags": {"x": "y"}}
    assert out["strData"] == "hello"
    # includingDefaultValueFields: an empty meta prints its defaults
    out = rt(C, {"meta": {}, "strData": ""})
    assert out["meta"] == {"puid": "", "tags": {}, "routing": {}, "requestPath": {}, "metrics": []}
    assert out["strData"] == ""


def test_bindata_and_jsondata(C):
    raw = bytes(range(256))
    out = rt(C, {"binData": base64.b64encode(raw).decode()})
    assert base64.b64decode(out["binData"]) == raw
    jd = {"a": [1, {"b": None}], "s": "x\n\"y\"", "u": "é中"}
    out = rt(C, {"jsonData": jd})
    assert out["jsonData"] == {"a": [1.0, {"b": None}], "s": "x\n\"y\"", "u": "é中"}


def test_status_roundtrip(C):
    out = rt(C, {"status": {"code": 203, "info": "i", "reason": "r", "status": "FAILURE"}})
    assert out["status"] == {"code": 203, "info": "i", "reason": "r", "status": "FAILURE"}


@pytest.mark.parametrize("bad", ['{"data":{"ndarray":[1]}, "strData":"x"}', '{"foo":1}', '{"data":{"tensor":1}}',
                                 '{"meta":{"routing":{"a":"x"}}}', '[1,2', '{"data":{"ndarray":[1],"tensor":{}}}'])
def test_invalid_json_rejected(C, bad):
    with pytest.raises(Exception):
        C.json_roundtrip(bad)


def test_protobuf_roundtrip(C):
    msg = {"status": {"code": 1, "info": "i", "reason": "", "status": "SUCCESS"},
           "meta": {"puid": "p", "tags": {"a": [1, "s", None, True, {"x": 2}]}, "routing": {"r": -1},
                    "requestPath": {"n": "img"}, "metrics": [{"key": "k", "type": "TIMER", "value": 22.5}]},
           "data": {"names": ["x"], "tensor": {"shape": [3, 2], "values": [1, 2, 3, 4, 5, 6]}}}
    pb = C.json_to_pb(json.dumps(msg))
    back = json.loads(C.pb_to_json(pb))
    assert back["data"]["tensor"] == {"shape": [3, 2], "values": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]}
    assert back["meta"]["routing"] == {"r": -1}
    assert back["meta"]["tags"]["a"] == [1.0, "s", None, True, {"x": 2.0}]
    assert back["meta"]["metrics"][0]["type"] == "TIMER"
    for payload in ({"strData": "s"}, {"binData": base64.b64encode(b"\x00\x01").decode()},
                    {"jsonData": {"k": [1, 2]}}, {"data": {"ndarray": [[1, 2], [3, 4]]}}):
        assert json.loads(C.pb_to_json(C.json_to_pb(json.dumps(payload)))) == rt(C, payload)


def test_protobuf_matches_python_protobuf_wire(C):
    """Our encoder/decoder agree with google.protobuf's Struct/Value encoding."""
    from google.protobuf import struct_pb2

    lv = struct_pb2.ListValue()
    lv.extend([1.0, "a", True])
    # DefaultData{ndarray=3} inside SeldonMessage{data=3}: build by hand
    inner = b"\x1a" + bytes([len(lv.SerializeToString())]) + lv.SerializeToString()
    wire = b"\x1a" + bytes([len(inner)]) + inner
    out = json.loads(C.pb_to_json(wire))
    assert out["data"]["ndarray"] == [1.0, "a", True]


def test_feedback_and_list_codecs(C):
    fb = {"request": {"data": {"ndarray": [[1.0]]}}, "response": {"meta": {"routing": {"r": 1}}}, "reward": 0.5,
          "truth": {"data": {"ndarray": [[0.0]]}}}
    back = json.loads(C.feedback_pb_to_json(C.feedback_json_to_pb(json.dumps(fb))))
    assert back["reward"] == 0.5 and back["response"]["meta"]["routing"] == {"r": 1}
    lst = {"seldonMessages": [{"strData": "a"}, {"data": {"tensor": {"shape": [1], "values": [2]}}}]}
    back = json.loads(C.list_pb_to_json(C.list_json_to_pb(json.dumps(lst))))
    assert back["seldonMessages"][0]["strData"] == "a"


def test_tftensor_dense_views(C):
    from seldon_core_amd.serving.codec import array_to_tftensor, tftensor_to_array

    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    t = array_to_tftensor(a)
    np.testing.assert_array_equal(tftensor_to_array(t), a)
    shape, vals = C.dense_of(json.dumps({"data": {"tftensor": t}}))
    assert shape == [2, 3] and vals == list(map(float, range(6)))
    shape, vals = C.dense_of(json.dumps({"data": {"tftensor": {"dtype": "DT_DOUBLE", "tensorShape": {
        "dim": [{"size": "2"}]}, "doubleVal": [1.5, 2.5]}}}))
    assert shape == [2] and vals == [1.5, 2.5]
    with pytest.raises(Exception):
        C.dense_of(json.dumps({"data": {"ndarray": [[1, 2], [3]]}}))


def test_number_formatting(C):
    vals = [0.1, 1e-300, 123456789.125, 1e22, -0.0, 5e-324, 2 ** 53]
    out = rt(C, {"data": {"tensor": {"shape": [len(vals)], "values": vals}}})
    assert out["data"]["tensor"]["values"] == vals


def test_tftensor_enum_number_dtype():
    """protobuf JSON may carry the DataType as its enum number (types.proto)."""
    from seldon_core_amd.serving.codec import tftensor_to_array

    shape = {"dim": [{"size": "2"}]}
    assert tftensor_to_array({"dtype": 2, "tensorShape": shape, "doubleVal": [1.5, 2.5]}).dtype == np.float64
    assert tftensor_to_array({"dtype": 9, "tensorShape": shape, "int64Val": ["3", "4"]}).tolist() == [3, 4]
    assert tftensor_to_array({"dtype": 1, "tensorShape": shape, "floatVal": [1, 2]}).dtype == np.float32
