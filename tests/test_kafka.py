"""Kafka prediction stream (reference kafka/tests/src/read_predictions.py).

No broker ships in this image, so a fake broker below speaks Metadata v1 /
Produce v3 / Fetch v4 from the protocol spec and keeps RecordBatches as the
producer sent them, assigning offsets like a partition leader.  Broker parity
is unpinned; the CRC-32C is pinned by its published check value."""
import json
import socket
import socketserver
import struct
import threading
import time
import urllib.request

import pytest

from seldon_core_amd import request_logger
from seldon_core_amd.proto import prediction_pb2
from seldon_core_amd.utils import kafka


class FakeBroker:
    def __init__(self, partitions=1):
        self.logs = {}  # (topic, partition) -> [bytes batches]
        self.next_off = {}
        self.partitions = partitions
        self.requests = []
        broker = self

        class H(socketserver.BaseRequestHandler):
            def handle(self):
                s = self.request
                while True:
                    hdr = self._read(s, 4)
                    if not hdr:
                        return
                    req = self._read(s, struct.unpack(">i", hdr)[0])
                    out = broker.dispatch(req)
                    if out is not None:
                        s.sendall(struct.pack(">i", len(out)) + out)

            @staticmethod
            def _read(s, n):
                b = bytearray()
                while len(b) < n:
                    c = s.recv(n - len(b))
                    if not c:
                        return None
                    b += c
                return bytes(b)

        self.srv = socketserver.ThreadingTCPServer(("127.0.0.1", 0), H)
        self.srv.daemon_threads = True
        self.port = self.srv.server_address[1]
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def dispatch(self, req):
        r = kafka._Reader(req)
        api, ver, corr = r.unpack(">hhi")
        r.string()  # client id
        self.requests.append((api, ver))
        head = struct.pack(">i", corr)
        if api == kafka.API_METADATA:
            assert ver == 1
            topics = r.array(r.string)
            body = struct.pack(">i", 1) + struct.pack(">i", 0) + kafka._str("127.0.0.1") + struct.pack(">i", self.port) + kafka._str(None)
            body += struct.pack(">i", 0) + struct.pack(">i", len(topics))
            for t in topics:
                body += struct.pack(">h", 0) + kafka._str(t) + struct.pack(">?", False) + struct.pack(">i", self.partitions)
                for p in range(self.partitions):
                    body += struct.pack(">hii", 0, p, 0) + struct.pack(">ii", 1, 0) + struct.pack(">ii", 1, 0)
            return head + body
        if api == kafka.API_PRODUCE:
            assert ver == 3
            r.string()
            acks, _timeout = r.unpack(">hi")
            resp = []
            for _ in range(r.unpack(">i")):
                topic = r.string()
                parts = []
                for _ in range(r.unpack(">i")):
                    p = r.unpack(">i")
                    batch = bytearray(r.bytes_())
                    recs = list(kafka.decode_batches(bytes(batch)))  # validates CRC
                    base = self.next_off.get((topic, p), 0)
                    batch[0:8] = struct.pack(">q", base)
                    self.logs.setdefault((topic, p), []).append(bytes(batch))
                    self.next_off[(topic, p)] = base + len(recs)
                    parts.append((p, base))
                resp.append((topic, parts))
            if acks == 0:
                return None
            body = struct.pack(">i", len(resp))
            for topic, parts in resp:
                body += kafka._str(topic) + struct.pack(">i", len(parts))
                for p, base in parts:
                    body += struct.pack(">ihqq", p, 0, base, -1)
            return head + body + struct.pack(">i", 0)
        if api == kafka.API_FETCH:
            assert ver == 4
            r.unpack(">iiiib")
            body = struct.pack(">i", 0)
            topics = []
            for _ in range(r.unpack(">i")):
                topic = r.string()
                parts = [r.unpack(">iqi") for _ in range(r.unpack(">i"))]
                topics.append((topic, parts))
            body += struct.pack(">i", len(topics))
            for topic, parts in topics:
                body += kafka._str(topic) + struct.pack(">i", len(parts))
                for p, off, _mx in parts:
                    data = b""
                    for b in self.logs.get((topic, p), []):
                        base, = struct.unpack_from(">q", b, 0)
                        n = struct.unpack_from(">i", b, 57)[0]
                        if base + n > off:
                            data += b
                    hw = self.next_off.get((topic, p), 0)
                    body += struct.pack(">ihqq", p, 0, hw, hw) + struct.pack(">i", -1) + kafka._bytes(data)
            return head + body
        raise AssertionError(f"unexpected api {api}")

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


@pytest.fixture
def broker():
    b = FakeBroker()
    yield b
    b.close()


def test_crc32c_check_value():
    assert kafka.crc32c(b"123456789") == 0xE3069283


@pytest.mark.parametrize("n", [0, 1, -1, 63, -64, 64, 300, -300, 2**31, -(2**40)])
def test_varint_roundtrip(n):
    b = kafka.varint(n)
    assert kafka.read_varint(b, 0) == (n, len(b))


def test_batch_roundtrip_and_corruption():
    recs = [(b"k1", b"v1", [("h", b"x")]), (None, b"", []), (b"k3", None, [])]
    buf = kafka.encode_batch(recs, base_offset=40, timestamp_ms=1234)
    out = list(kafka.decode_batches(buf))
    assert [(o, t, k, v, h) for o, t, k, v, h in out] == [
        (40, 1234, b"k1", b"v1", [("h", b"x")]), (41, 1234, None, b"", []), (42, 1234, b"k3", None, [])]
    bad = bytearray(buf)
    bad[-1] ^= 1
    with pytest.raises(kafka.CorruptBatch):
        list(kafka.decode_batches(bytes(bad)))
    assert list(kafka.decode_batches(buf[:-3])) == []  # partial trailing batch skipped


def test_produce_then_consume(broker):
    p = kafka.KafkaProducer(f"127.0.0.1:{broker.port}")
    assert p.send("preds", b"a", key=b"1") == 0
    assert p.send_batch("preds", [(None, b"b", []), (None, b"c", [])]) == 1
    c = kafka.KafkaConsumer(f"127.0.0.1:{broker.port}", "preds", 0, offset=2)
    got = c.poll()
    assert [(o, v) for o, _t, _k, v, _h in got] == [(2, b"c")]  # mid-batch seek
    assert c.poll() == []
    p.send("preds", b"d")
    assert [(o, v) for o, _t, _k, v, _h in c.poll()] == [(3, b"d")]
    p.close()
    c.close()
    assert (kafka.API_METADATA, 1) in broker.requests


def test_producer_round_robins_partitions():
    b = FakeBroker(partitions=3)
    try:
        p = kafka.KafkaProducer(f"127.0.0.1:{b.port}")
        for i in range(6):
            p.send("t", bytes([i]))
        assert sorted(k[1] for k in b.logs) == [0, 1, 2]
        assert all(len(v) == 2 for v in b.logs.values())
        p.close()
    finally:
        b.close()


def test_request_logger_publishes_request_response(broker, tmp_path):
    import io

    sink = request_logger.KafkaSink(f"127.0.0.1:{broker.port}", "predictions", linger_s=0.01)
    out = io.StringIO()
    srv = request_logger.serve("127.0.0.1", 0, out=out, sink=sink)
    port = srv.server_address[1]
    try:
        for i in range(5):
            pair = {"request": {"data": {"names": ["a", "b"], "ndarray": [[float(i), 2.0]]}},
                    "response": {"meta": {"puid": f"p{i}"}, "data": {"names": ["y"], "ndarray": [[float(i) * 10]]}}}
            req = urllib.request.Request(f"http://127.0.0.1:{port}/", data=json.dumps(pair).encode(),
                                         headers={"Content-Type": "application/json", "ce-type": "seldon.message.pair"})
            urllib.request.urlopen(req, timeout=5).read()
        t0 = time.time()
        while sink.sent < 5 and time.time() - t0 < 5:
            time.sleep(0.01)
        assert sink.sent == 5 and sink.dropped == 0
    finally:
        srv.shutdown()
        sink.close()
    c = kafka.KafkaConsumer(f"127.0.0.1:{broker.port}", "predictions")
    msgs = c.poll()
    c.close()
    assert [o for o, *_ in msgs] == list(range(5))
    for i, (_o, _t, key, value, headers) in enumerate(msgs):
        m = prediction_pb2.RequestResponse()
        m.ParseFromString(value)
        assert key == f"p{i}".encode()
        assert m.response.meta.puid == f"p{i}"
        assert m.request.data.ndarray.values[0].list_value.values[0].number_value == float(i)
        assert headers == [("content-type", b"application/x-protobuf")]


def test_sink_survives_broker_down():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    sink = request_logger.KafkaSink(f"127.0.0.1:{port}", "t", linger_s=0.0,
                                    producer=kafka.KafkaProducer(f"127.0.0.1:{port}", timeout=0.5))
    sink.publish({"request": {"data": {"ndarray": [[1]]}}})
    t0 = time.time()
    while sink.dropped == 0 and time.time() - t0 < 5:
        time.sleep(0.01)
    assert sink.dropped == 1
    sink.close()


def test_read_predictions_cli(broker, capsys):
    p = kafka.KafkaProducer(f"127.0.0.1:{broker.port}")
    m = prediction_pb2.RequestResponse()
    m.response.meta.puid = "xyz"
    p.send("preds", m.SerializeToString())
    p.close()
    assert kafka.main(["--kafka", f"127.0.0.1:{broker.port}", "--topic", "preds", "--max", "1"]) == 0
    line = capsys.readouterr().out.strip()
    assert line.startswith("0 ") and json.loads(line[2:])["response"]["meta"]["puid"] == "xyz"
