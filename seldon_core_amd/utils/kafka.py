"""Prediction stream over Kafka without a client library.

The reference ships Kafka/ZooKeeper manifests (``kafka/kafka.json``,
``helm-charts/seldon-core-kafka``) as a legacy prediction-stream sink, and a
reader that consumes ``RequestResponse`` protos from partition 0 of a topic
from offset 0 (``kafka/tests/src/read_predictions.py:1-29``).  No Kafka
package is importable here, so this module speaks the broker wire protocol
directly over a socket:

* ``Metadata`` v1 to find the partition leader,
* ``Produce`` v3 carrying a magic-2 ``RecordBatch`` (CRC-32C, zig-zag varint
  records) -- the oldest produce format Kafka 4.x still accepts,
* ``Fetch`` v4 (record batches, isolation level) for the reader.

Every request uses the non-flexible header v1 (api_key, api_version,
correlation_id, client_id); responses carry header v0.  Parity with a real
broker is unpinned (no broker in this image); the codec is pinned by the
CRC-32C check value and by round trips through the fake broker in
``tests/test_kafka.py``.

    python -m seldon_core_amd.utils.kafka --kafka localhost:9093 --topic predictions
"""
from __future__ import annotations

import argparse
import itertools
import socket
import struct
import sys
import threading
import time
from typing import Iterator, List, Optional, Sequence, Tuple

API_PRODUCE, API_FETCH, API_METADATA = 0, 1, 3

# ------------------------------------------------------------------ CRC-32C
_CRC32C = []
for _n in range(256):
    _c = _n
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC32C.append(_c)


def crc32c(data: bytes, crc: int = 0) -> int:
    """Castagnoli CRC (RecordBatch v2 checksum)."""
    crc ^= 0xFFFFFFFF
    tab = _CRC32C
    for b in data:
        crc = tab[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


# ------------------------------------------------------------------ varints
def _zz(n: int) -> int:
    return (n << 1) ^ (n >> 63)


def varint(n: int) -> bytes:
    u = _zz(n) & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while u >= 0x80:
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u)
    return bytes(out)


def read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = u = 0
    while True:
        b = buf[pos]
        pos += 1
        u |= (b & 0x7F) << shift
        if not b & 0x80:
            break
        shift += 7
    return (u >> 1) ^ -(u & 1), pos


def _vbytes(b: Optional[bytes]) -> bytes:
    return varint(-1) if b is None else varint(len(b)) + b


def _read_vbytes(buf: bytes, pos: int) -> Tuple[Optional[bytes], int]:
    n, pos = read_varint(buf, pos)
    if n < 0:
        return None, pos
    return bytes(buf[pos:pos + n]), pos + n


# ------------------------------------------------------------ record batch
Record = Tuple[Optional[bytes], Optional[bytes], Sequence[Tuple[str, bytes]]]  # key, value, headers


def encode_batch(records: Sequence[Record], base_offset: int = 0, timestamp_ms: Optional[int] = None) -> bytes:
    """Magic-2 RecordBatch, uncompressed, non-transactional."""
    ts = int(time.time() * 1000) if timestamp_ms is None else int(timestamp_ms)
    body = bytearray()
    for i, (key, value, headers) in enumerate(records):
        r = bytearray(b"\x00")  # attributes
        r += varint(0) + varint(i) + _vbytes(key) + _vbytes(value) + varint(len(headers))
        for hk, hv in headers:
            r += _vbytes(hk.encode()) + _vbytes(hv)
        body += varint(len(r)) + r
    n = len(records)
    # attributes .. records: the CRC-32C covered part
    tail = struct.pack(">hiqqqhii", 0, max(n - 1, 0), ts, ts, -1, -1, -1, n) + bytes(body)
    after_len = struct.pack(">ib", -1, 2) + struct.pack(">I", crc32c(tail)) + tail
    return struct.pack(">qi", base_offset, len(after_len)) + after_len


class CorruptBatch(ValueError):
    pass


def decode_batches(buf: bytes) -> Iterator[Tuple[int, int, Optional[bytes], Optional[bytes], List[Tuple[str, bytes]]]]:
    """Yield (offset, timestamp_ms, key, value, headers); a trailing partial batch is skipped."""
    pos = 0
    while pos + 12 <= len(buf):
        base_offset, blen = struct.unpack_from(">qi", buf, pos)
        end = pos + 12 + blen
        if end > len(buf):
            break  # partial batch at the end of a fetch (max_bytes cut)
        magic = buf[pos + 16]
        if magic != 2:
            raise CorruptBatch(f"unsupported record batch magic {magic}")
        (crc,) = struct.unpack_from(">I", buf, pos + 17)
        if crc32c(bytes(buf[pos + 21:end])) != crc:
            raise CorruptBatch(f"CRC-32C mismatch in batch at offset {base_offset}")
        attrs, _last, base_ts, _max_ts, _pid, _pep, _seq, n = struct.unpack_from(">hiqqqhii", buf, pos + 21)
        if attrs & 0x7:
            raise CorruptBatch("compressed record batches are not supported")
        p = pos + 21 + struct.calcsize(">hiqqqhii")
        for _ in range(n):
            rlen, p = read_varint(buf, p)
            rend = p + rlen
            p += 1  # record attributes
            ts_delta, p = read_varint(buf, p)
            off_delta, p = read_varint(buf, p)
            key, p = _read_vbytes(buf, p)
            value, p = _read_vbytes(buf, p)
            nh, p = read_varint(buf, p)
            headers = []
            for _h in range(nh):
                hk, p = _read_vbytes(buf, p)
                hv, p = _read_vbytes(buf, p)
                headers.append(((hk or b"").decode(), hv))
            p = rend
            yield base_offset + off_delta, base_ts + ts_delta, key, value, headers
        pos = end


# ------------------------------------------------------------ wire helpers
def _str(s: Optional[str]) -> bytes:
    if s is None:
        return struct.pack(">h", -1)
    b = s.encode()
    return struct.pack(">h", len(b)) + b


def _bytes(b: Optional[bytes]) -> bytes:
    return struct.pack(">i", -1) if b is None else struct.pack(">i", len(b)) + b


class _Reader:
    def __init__(self, buf: bytes):
        self.buf, self.pos = buf, 0

    def unpack(self, fmt: str):
        v = struct.unpack_from(fmt, self.buf, self.pos)
        self.pos += struct.calcsize(fmt)
        return v if len(v) > 1 else v[0]

    def string(self) -> Optional[str]:
        n = self.unpack(">h")
        if n < 0:
            return None
        s = self.buf[self.pos:self.pos + n].decode()
        self.pos += n
        return s

    def bytes_(self) -> Optional[bytes]:
        n = self.unpack(">i")
        if n < 0:
            return None
        b = bytes(self.buf[self.pos:self.pos + n])
        self.pos += n
        return b

    def array(self, item):
        n = self.unpack(">i")
        return [] if n < 0 else [item() for _ in range(n)]


class KafkaError(RuntimeError):
    def __init__(self, code: int, where: str):
        super().__init__(f"kafka error {code} in {where}")
        self.code = code


class _Conn:
    def __init__(self, host: str, port: int, client_id: str, timeout: float):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.client_id = client_id
        self._corr = itertools.count(1)
        self.lock = threading.Lock()

    def _recv_exact(self, n: int) -> bytes:
        out = bytearray()
        while len(out) < n:
            chunk = self.sock.recv(n - len(out))
            if not chunk:
                raise ConnectionError("kafka broker closed the connection")
            out += chunk
        return bytes(out)

    def call(self, api_key: int, version: int, body: bytes, expect_reply: bool = True) -> Optional[_Reader]:
        with self.lock:
            corr = next(self._corr)
            req = struct.pack(">hhi", api_key, version, corr) + _str(self.client_id) + body
            self.sock.sendall(struct.pack(">i", len(req)) + req)
            if not expect_reply:
                return None
            (size,) = struct.unpack(">i", self._recv_exact(4))
            resp = self._recv_exact(size)
        r = _Reader(resp)
        if r.unpack(">i") != corr:
            raise ConnectionError("kafka correlation id mismatch")
        return r

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


def _parse_endpoint(ep: str) -> Tuple[str, int]:
    host, _, port = ep.rpartition(":")
    return (host or "localhost"), int(port or 9092)


class _Client:
    def __init__(self, bootstrap: str, client_id: str, timeout: float):
        self.bootstrap = [_parse_endpoint(e.strip()) for e in bootstrap.split(",") if e.strip()]
        self.client_id, self.timeout = client_id, timeout
        self.conns = {}
        self.leaders = {}  # (topic, partition) -> (host, port)
        self.partitions = {}  # topic -> [partition ids]

    def _conn(self, addr: Tuple[str, int]) -> _Conn:
        c = self.conns.get(addr)
        if c is None:
            c = self.conns[addr] = _Conn(addr[0], addr[1], self.client_id, self.timeout)
        return c

    def metadata(self, topic: str) -> None:
        last = None
        for addr in self.bootstrap:
            try:
                r = self._conn(addr).call(API_METADATA, 1, struct.pack(">i", 1) + _str(topic))
                break
            except OSError as e:
                self.conns.pop(addr, None)
                last = e
        else:
            raise ConnectionError(f"no kafka bootstrap broker reachable: {last}")
        brokers = {}
        for node, host, port, _rack in r.array(lambda: (r.unpack(">i"), r.string(), r.unpack(">i"), r.string())):
            brokers[node] = (host, port)
        r.unpack(">i")  # controller id

        def part():
            err, idx, leader = r.unpack(">hii")
            r.array(lambda: r.unpack(">i"))
            r.array(lambda: r.unpack(">i"))
            return err, idx, leader

        for terr, name, _internal, parts in r.array(lambda: (r.unpack(">h"), r.string(), r.unpack(">?"), r.array(part))):
            if terr:
                raise KafkaError(terr, f"metadata({name})")
            self.partitions[name] = sorted(p[1] for p in parts)
            for perr, idx, leader in parts:
                if leader in brokers:
                    self.leaders[(name, idx)] = brokers[leader]

    def leader(self, topic: str, partition: int) -> _Conn:
        if (topic, partition) not in self.leaders:
            self.metadata(topic)
        if (topic, partition) not in self.leaders:
            raise KafkaError(3, f"no leader for {topic}/{partition}")  # UNKNOWN_TOPIC_OR_PARTITION
        return self._conn(self.leaders[(topic, partition)])

    def close(self):
        for c in self.conns.values():
            c.close()
        self.conns.clear()


class KafkaProducer(_Client):
    """Synchronous producer: one RecordBatch per ``send_batch`` call."""

    def __init__(self, bootstrap: str, client_id: str = "seldon-amd", acks: int = 1, timeout: float = 10.0):
        super().__init__(bootstrap, client_id, timeout)
        self.acks = acks
        self._rr = itertools.count()

    def send_batch(self, topic: str, records: Sequence[Record], partition: Optional[int] = None) -> int:
        """Append records; returns the base offset the broker assigned (-1 with acks=0)."""
        if partition is None:
            if topic not in self.partitions:
                self.metadata(topic)
            parts = self.partitions.get(topic) or [0]
            partition = parts[next(self._rr) % len(parts)]
        conn = self.leader(topic, partition)
        batch = encode_batch(records)
        body = (_str(None) + struct.pack(">hi", self.acks, int(self.timeout * 1000)) + struct.pack(">i", 1) + _str(topic)
                + struct.pack(">i", 1) + struct.pack(">i", partition) + _bytes(batch))
        r = conn.call(API_PRODUCE, 3, body, expect_reply=self.acks != 0)
        if r is None:
            return -1
        base = -1
        for _name, parts in r.array(lambda: (r.string(), r.array(lambda: r.unpack(">ihqq")))):
            for _idx, err, off, _ts in parts:
                if err:
                    self.leaders.pop((topic, partition), None)  # NOT_LEADER etc.: refresh next time
                    raise KafkaError(err, f"produce({topic}/{partition})")
                base = off
        return base

    def send(self, topic: str, value: bytes, key: Optional[bytes] = None, headers=(), partition: Optional[int] = None) -> int:
        return self.send_batch(topic, [(key, value, list(headers))], partition)


class KafkaConsumer(_Client):
    """Reads one partition from an offset (the reference reader's seek(partition, 0))."""

    def __init__(self, bootstrap: str, topic: str, partition: int = 0, offset: int = 0, client_id: str = "seldon-amd",
                 max_bytes: int = 1 << 20, max_wait_ms: int = 500, timeout: float = 10.0):
        super().__init__(bootstrap, client_id, timeout)
        self.topic, self.partition, self.offset = topic, partition, offset
        self.max_bytes, self.max_wait_ms = max_bytes, max_wait_ms

    def poll(self) -> List[Tuple[int, int, Optional[bytes], Optional[bytes], List[Tuple[str, bytes]]]]:
        conn = self.leader(self.topic, self.partition)
        body = (struct.pack(">iiiib", -1, self.max_wait_ms, 1, self.max_bytes, 0) + struct.pack(">i", 1)
                + _str(self.topic) + struct.pack(">i", 1) + struct.pack(">iqi", self.partition, self.offset, self.max_bytes))
        r = conn.call(API_FETCH, 4, body)
        r.unpack(">i")  # throttle
        out = []
        for _t in range(r.unpack(">i")):
            r.string()
            for _p in range(r.unpack(">i")):
                _idx, err, _hw, _lso = r.unpack(">ihqq")
                r.array(lambda: r.unpack(">qq"))
                records = r.bytes_()
                if err:
                    raise KafkaError(err, f"fetch({self.topic}/{self.partition})")
                for rec in decode_batches(records or b""):
                    if rec[0] >= self.offset:  # a batch may start before the requested offset
                        out.append(rec)
        if out:
            self.offset = out[-1][0] + 1
        return out

    def __iter__(self):
        while True:
            yield from self.poll()


# ------------------------------------------------------------- CLI reader
def main(argv=None) -> int:
    """Print RequestResponse protos from a topic (reference read_predictions.py)."""
    from ..proto import prediction_pb2
    from google.protobuf import json_format

    ap = argparse.ArgumentParser(prog="read_predictions")
    ap.add_argument("--kafka", default="localhost:9093", help="kafka endpoint")
    ap.add_argument("--topic", required=True, help="kafka topic")
    ap.add_argument("--partition", type=int, default=0)
    ap.add_argument("--max", type=int, default=0, help="stop after this many messages (0 = follow)")
    args = ap.parse_args(argv)
    c = KafkaConsumer(args.kafka, args.topic, args.partition, 0)
    n = 0
    try:
        for off, _ts, _key, value, _h in c:
            m = prediction_pb2.RequestResponse()
            m.ParseFromString(value or b"")
            print(off, json_format.MessageToJson(m, indent=None), flush=True)
            n += 1
            if args.max and n >= args.max:
                break
    finally:
        c.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
