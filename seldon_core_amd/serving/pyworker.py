"""Worker process of a Python component's process pool (the analogue of the
reference's gunicorn workers, python/seldon_core/microservice.py:153-174).

Started by ``PythonUnit.start_pool`` as a fresh interpreter with one end of a
Unix socketpair.  The first frame carries the pickled component; every later
frame is one (possibly stacked) call from the native unit
(csrc/bindings/py_unit.h: PoolFrame): dense requests arrive as raw fp64 rows
plus a small JSON text (feature names, request meta, data kind), everything
else as ``<node json>\\n<SeldonMessage JSON>``.  The component's own
state is the parent's (pickled after ``load()``), as when gunicorn forks its
workers from a loaded app.
"""
from __future__ import annotations

import json
import pickle
import socket
import sys
import traceback

import numpy as np

from .adapter import OP_INIT, PythonUnit, recv_frame, send_frame

OPS = {1: "predict", 2: "transform_input", 3: "transform_output", 4: "route", 5: "aggregate", 6: "send_feedback"}


def serve(fd: int) -> None:
    sock = socket.socket(fileno=fd)
    op, _, _, _, blob = recv_frame(sock)
    if op != OP_INIT:
        raise SystemExit("first frame must be the component")
    try:
        payload = pickle.loads(blob)
        obj = payload["obj"]  # already load()ed in the parent; its state travels in the pickle
        unit = PythonUnit(obj, payload["unit_type"], payload["name"], lock=False)
        send_frame(sock, 0, b"", b"ok")
    except Exception:  # noqa: BLE001
        send_frame(sock, 3, b"", traceback.format_exc().encode())
        return
    while True:
        try:
            op, flags, shape, x, text = recv_frame(sock)
        except (EOFError, ConnectionError, OSError):
            return
        method = OPS.get(op)
        try:
            if method is None:
                raise ValueError(f"unknown op {op}")
            if flags & 1:
                info = json.loads(text)
                X = np.frombuffer(x, dtype=np.float64).reshape(shape)
                meta = info.get("meta")
                res = unit.call_dense(method, X, info.get("names") or [], json.dumps(meta) if meta else None,
                                      info.get("kind", "tensor"))
                if res[0] == 0:
                    _, y, names, meta_all, meta_first = res
                    out = json.dumps({"names": names, "meta": json.loads(meta_all) if meta_all else None,
                                      "meta_first": json.loads(meta_first) if meta_first else None})
                    send_frame(sock, 0, y.tobytes(), out.encode(), shape=y.shape)
                else:
                    send_frame(sock, 1, b"", res[1].encode())
            else:
                node_json, _, msg = text.decode().partition("\n")
                out = unit.call_json(method, msg, json.loads(node_json))
                if isinstance(out, tuple):  # a raw hook's numeric array: binary frame, no JSON
                    y, names, kind, meta = out
                    info = json.dumps({"names": names, "meta": json.loads(meta) if meta else None,
                                       "meta_first": None, "kind": kind})
                    send_frame(sock, 0, y.tobytes(), info.encode(), shape=y.shape)
                else:
                    send_frame(sock, 1, b"", (out or "").encode())
        except Exception as e:  # noqa: BLE001
            try:
                reply = unit.error_reply(e)  # the component's own status + body (op 4)
                if reply is not None:
                    send_frame(sock, 4, b"", json.dumps({"status": reply[0], "body": reply[1],
                                                         "info": reply[2]}).encode())
                else:
                    send_frame(sock, 3, b"", f"{type(e).__name__}: {e}".encode())
            except OSError:
                return


if __name__ == "__main__":
    serve(int(sys.argv[1]))
