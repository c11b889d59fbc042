"""Model-artifact fetch over the object-store HTTP APIs (reference
python/seldon_core/storage.py:36-160), against an in-process fake S3 / GCS /
Azure endpoint.  SigV4 is pinned to AWS's published signing example."""
import json
import os
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from seldon_core_amd.utils.storage import Storage, sigv4_headers, sigv4_signing_key

OBJECTS = {"models/iris/model.joblib": b"JOBLIB" * 100, "models/iris/meta/info.json": b'{"a": 1}',
           "models/iris/sub/dir/x.bin": bytes(range(256)), "other/y": b"nope"}
AK, SK = "AKIDTEST", "secret/KEY+test"


def test_sigv4_matches_aws_documented_example():
    # "Signature Version 4 signing process" example (IAM ListUsers).
    key = sigv4_signing_key("wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY", "20150830", "us-east-1", "iam")
    assert key.hex() == "c4afb1cc5771d871763a393e44b703571b55cc28424d1a5e86da6ed3c154a4b9"
    h = sigv4_headers("GET", "https://iam.amazonaws.com/?Action=ListUsers&Version=2010-05-08",
                      access_key="AKIDEXAMPLE", secret_key="wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY",
                      region="us-east-1", service="iam",
                      headers={"Content-Type": "application/x-www-form-urlencoded; charset=utf-8"},
                      amz_date="20150830T123600Z", sign_payload_header=False)
    assert h["Authorization"].endswith(
        "Signature=5d672d79c15b13162d9279b0855cfba6789a8edb4c82c400e06b5924a6f2b5d7")
    assert "SignedHeaders=content-type;host;x-amz-date" in h["Authorization"]


class _Fake(BaseHTTPRequestHandler):
    seen = []

    def log_message(self, *a):
        pass

    def _send(self, code, body, ctype="application/octet-stream"):
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_GET(self):
        u = urllib.parse.urlsplit(self.path)
        q = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        parts = [urllib.parse.unquote(p) for p in u.path.split("/")[1:]]
        _Fake.seen.append(self.path)
        if parts[0] == "storage":  # GCS JSON API: /storage/v1/b/<bucket>/o[/<name>]
            if len(parts) == 5:
                names = sorted(k for k in OBJECTS if k.startswith(q.get("prefix", "")))
                start = int(q.get("pageToken", "0"))
                page = {"items": [{"name": n} for n in names[start:start + 2]]}
                if start + 2 < len(names):
                    page["nextPageToken"] = str(start + 2)
                return self._send(200, json.dumps(page).encode(), "application/json")
            assert q.get("alt") == "media"
            return self._send(200, OBJECTS[parts[5]])
        if parts[0] == "acct":  # Azure: /acct/<container>[/<blob>]
            if len(parts) == 2:
                assert q["restype"] == "container" and q["comp"] == "list"
                names = sorted(k for k in OBJECTS if k.startswith(q.get("prefix", "")))
                start = int(q.get("marker", "0") or 0)
                xml = "<?xml version='1.0'?><EnumerationResults><Blobs>" + "".join(
                    f"<Blob><Name>{n}</Name></Blob>" for n in names[start:start + 2]) + "</Blobs>"
                xml += f"<NextMarker>{start + 2 if start + 2 < len(names) else ''}</NextMarker></EnumerationResults>"
                return self._send(200, xml.encode(), "application/xml")
            return self._send(200, OBJECTS["/".join(parts[2:])])
        # S3 path-style: /<bucket>[/<key>], SigV4-signed.
        auth = self.headers.get("Authorization", "")
        assert auth.startswith(f"AWS4-HMAC-SHA256 Credential={AK}/")
        want = sigv4_headers("GET", f"http://{self.headers['Host']}{self.path}", access_key=AK, secret_key=SK,
                             region="eu-west-1", amz_date=self.headers["x-amz-date"])
        if want["Authorization"] != auth:
            return self._send(403, b"<Error>SignatureDoesNotMatch</Error>")
        if len(parts) == 1 or (len(parts) == 2 and parts[1] == ""):
            names = sorted(k for k in OBJECTS if k.startswith(q.get("prefix", "")))
            start = int(q.get("continuation-token", "0"))
            ns = "http://s3.amazonaws.com/doc/2006-03-01/"
            more = start + 2 < len(names)
            xml = f"<ListBucketResult xmlns='{ns}'>" + "".join(
                f"<Contents><Key>{n}</Key></Contents>" for n in names[start:start + 2])
            xml += f"<IsTruncated>{'true' if more else 'false'}</IsTruncated>"
            if more:
                xml += f"<NextContinuationToken>{start + 2}</NextContinuationToken>"
            return self._send(200, (xml + "</ListBucketResult>").encode(), "application/xml")
        return self._send(200, OBJECTS["/".join(parts[1:])])


@pytest.fixture(scope="module")
def fake():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Fake)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield f"127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()


def _check_tree(d, rel_root=""):
    assert open(os.path.join(d, rel_root, "model.joblib"), "rb").read() == OBJECTS["models/iris/model.joblib"]
    assert open(os.path.join(d, rel_root, "meta/info.json"), "rb").read() == b'{"a": 1}'
    assert open(os.path.join(d, rel_root, "sub/dir/x.bin"), "rb").read() == bytes(range(256))
    assert not os.path.exists(os.path.join(d, rel_root, "y"))


def test_s3_download_sigv4_paginated(fake, monkeypatch, tmp_path):
    monkeypatch.setenv("S3_ENDPOINT", f"http://{fake}")
    monkeypatch.setenv("AWS_ACCESS_KEY_ID", AK)
    monkeypatch.setenv("AWS_SECRET_ACCESS_KEY", SK)
    monkeypatch.setenv("AWS_REGION", "eu-west-1")
    out = Storage.download("s3://bucket/models/iris", str(tmp_path))
    assert out == str(tmp_path)
    _check_tree(out)
    monkeypatch.setenv("AWS_SECRET_ACCESS_KEY", "wrong")
    with pytest.raises(RuntimeError, match="403"):
        Storage.download("s3://bucket/models/iris", str(tmp_path / "x"))


def test_gcs_download(fake, monkeypatch, tmp_path):
    monkeypatch.setenv("STORAGE_EMULATOR_HOST", f"http://{fake}")
    out = Storage.download("gs://bucket/models/iris")  # no out_dir -> temp dir
    _check_tree(out)


def test_azure_blob_download_keeps_blob_names(fake, monkeypatch, tmp_path):
    monkeypatch.setenv("AZURE_BLOB_ENDPOINT", f"http://{fake}/acct")
    out = Storage.download("https://acct.blob.core.windows.net/container/models/iris", str(tmp_path))
    _check_tree(out, "models/iris")


def test_local_and_pvc_semantics(tmp_path, monkeypatch):
    src = tmp_path / "m"
    (src / "d").mkdir(parents=True)
    (src / "a.txt").write_text("A")
    (src / "d" / "b.txt").write_text("B")
    assert Storage.download(f"file://{src}") == str(src)
    out = Storage.download(str(src), str(tmp_path / "out"))
    assert os.path.islink(os.path.join(out, "a.txt")) and open(os.path.join(out, "d", "b.txt")).read() == "B"
    monkeypatch.setenv("SELDON_PVC_ROOT", str(tmp_path))
    assert Storage.download("pvc://m") == str(src)
    with pytest.raises(FileNotFoundError):
        Storage.download("file:///nonexistent/path")
    with pytest.raises(RuntimeError, match="Cannot recognize"):
        Storage.download("ftp://x/y", str(tmp_path / "z"))


def test_mirror_short_circuits_remote(tmp_path, monkeypatch):
    (tmp_path / "bucket" / "models").mkdir(parents=True)
    (tmp_path / "bucket" / "models" / "w.bin").write_bytes(b"W")
    monkeypatch.setenv("SELDON_STORAGE_MIRROR", str(tmp_path))
    out = Storage.download("s3://bucket/models", str(tmp_path / "o"))
    assert open(os.path.join(out, "w.bin"), "rb").read() == b"W"
