"""REST fast path for dense ndarray requests (csrc/core/message.cc:
fast_dense_message) must produce exactly the message the general JSON
parser + message_from_json produce, and decline everything else."""

import pytest

import seldon_core_amd as sca

# through the loader (torch first: one HIP runtime in the process); a bare
# `import seldon_core_amd._C` here, at collection time, made every later GPU
# test in the session see 0 devices
_C = sca.native()

ACCEPT = [
    '{"data":{"names":["a","b","c","d"],"ndarray":[[5.1,3.5,1.4,0.2]]}}',
    '{"data":{"ndarray":[[5.1,3.5,1.4,0.2],[1,2,3,4]],"names":["a","b","c","d"]}}',
    ' { "meta" : { } , "data" : { "ndarray" : [ [ -1e-3 , 2E5 , +7 , 0.1 ] ] } } ',
    '{"data":{"names":[],"ndarray":[[1]]}}',
    '{"data":{"ndarray":[[1.0000000000000002, 123456789012345678901234567890]]}}',
    '{"data":{"names":["été"],"ndarray":[[3]]}}',
]
DECLINE = [
    '{"data":{"ndarray":[1,2,3]}}',                       # 1-D
    '{"data":{"ndarray":[[1,2],[3]]}}',                   # ragged
    '{"data":{"ndarray":[]}}',                            # empty
    '{"data":{"ndarray":[["a"]]}}',                       # non-numeric
    '{"data":{"ndarray":[[NaN]]}}',                       # literal
    '{"data":{"names":["a\\"b"],"ndarray":[[1]]}}',       # escape
    '{"data":{"tensor":{"shape":[1,1],"values":[1]}}}',   # other oneof
    '{"meta":{"puid":"x"},"data":{"ndarray":[[1]]}}',     # non-empty meta
    '{"data":{"ndarray":[[1]]},"data":{"ndarray":[[2]]}}',  # duplicate key
    '{"strData":"x"}',
    '{"data":{"ndarray":[[1]]}} x',                       # trailing garbage
    '{"data":{"ndarray":[[1]],"foo":1}}',                 # unknown field
]

@pytest.mark.parametrize("text", ACCEPT)
def test_fast_path_matches_general_parser(text):
    got = _C.json_fast_roundtrip(text)
    assert got is not None, text
    js, pb = got
    assert js == _C.json_roundtrip(text)
    assert pb == _C.json_to_pb(text)

@pytest.mark.parametrize("text", DECLINE)
def test_fast_path_declines(text):
    assert _C.json_fast_roundtrip(text) is None
