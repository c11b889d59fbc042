"""Model artifact fetch (reference python/seldon_core/storage.py:36-160 and the
operator's model-initializer init container, operator/controllers/
model_initializer_injector.go:65-209).

Same URI schemes and directory semantics as the reference, without its SDKs
(minio / google-cloud-storage / azure-storage are not shipped here): each
object store is spoken to over its plain HTTP API with the standard library.

* ``s3://bucket/prefix`` -- S3 / MinIO ListObjectsV2 + GetObject, path-style,
  AWS Signature V4 (``AWS_ACCESS_KEY_ID`` / ``AWS_SECRET_ACCESS_KEY`` /
  ``AWS_SESSION_TOKEN``; anonymous when unset).  Endpoint from ``S3_ENDPOINT``
  (reference ``_create_minio_client``: scheme decides TLS, else ``USE_SSL``),
  region from ``AWS_REGION`` (default ``us-east-1``).
* ``gs://bucket/prefix`` -- GCS JSON API list + ``alt=media`` download;
  bearer token from ``GOOGLE_OAUTH_ACCESS_TOKEN`` (anonymous otherwise, like
  the reference's ``create_anonymous_client`` fallback); endpoint override
  ``STORAGE_EMULATOR_HOST``.
* ``https://<account>.blob.core.windows.net/<container>/<prefix>`` -- Azure
  Blob list (``restype=container&comp=list``) + GET; optional SAS token from
  ``AZURE_STORAGE_SAS_TOKEN``; endpoint override ``AZURE_BLOB_ENDPOINT``
  (e.g. an Azurite ``http://host:port/<account>``).
* ``file://`` / local paths -- returned in place, or their entries symlinked
  into ``out_dir`` (reference ``_download_local``).
* ``pvc://<claim>/<path>`` -- ``$SELDON_PVC_ROOT/<claim>/<path>`` (default
  ``/mnt``), the init container's volume mount.

``SELDON_STORAGE_MIRROR=<dir>`` short-circuits every remote scheme to a local
mirror laid out as ``<dir>/<bucket>/<key>`` (air-gapped clusters).
"""
from __future__ import annotations

import datetime as _dt
import glob
import hashlib
import hmac
import json
import logging
import os
import re
import shutil
import tempfile
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET

_LOCAL_PREFIX = "file://"
_GCS_PREFIX = "gs://"
_S3_PREFIX = "s3://"
_PVC_PREFIX = "pvc://"
_BLOB_RE = r"https://(.+?)\.blob\.core\.windows\.net/(.+)"
_CHUNK = 1 << 20

log = logging.getLogger(__name__)


# ------------------------------------------------------------ AWS SigV4
def _sha256_hex(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_signing_key(secret: str, date: str, region: str, service: str) -> bytes:
    k = _hmac(("AWS4" + secret).encode(), date)
    k = _hmac(k, region)
    k = _hmac(k, service)
    return _hmac(k, "aws4_request")


def _uri_encode(s: str, safe: str = "-_.~") -> str:
    return urllib.parse.quote(s, safe=safe)


def sigv4_headers(method: str, url: str, *, access_key: str, secret_key: str, region: str, service: str = "s3",
                  headers: dict | None = None, payload: bytes = b"", amz_date: str | None = None,
                  session_token: str | None = None, sign_payload_header: bool = True) -> dict:
    """Return ``headers`` plus ``x-amz-date`` / ``Authorization`` (and
    ``x-amz-content-sha256`` for S3) signed with AWS Signature Version 4."""
    u = urllib.parse.urlsplit(url)
    amz_date = amz_date or _dt.datetime.now(_dt.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
    date = amz_date[:8]
    payload_hash = _sha256_hex(payload)
    h = {k.lower(): " ".join(str(v).split()) for k, v in (headers or {}).items()}
    h["host"] = u.netloc
    h["x-amz-date"] = amz_date
    if sign_payload_header:
        h["x-amz-content-sha256"] = payload_hash
    if session_token:
        h["x-amz-security-token"] = session_token
    signed = ";".join(sorted(h))
    canon_headers = "".join(f"{k}:{h[k]}\n" for k in sorted(h))
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canon_query = "&".join(f"{_uri_encode(k)}={_uri_encode(v)}" for k, v in sorted(q))
    canon_path = _uri_encode(urllib.parse.unquote(u.path or "/"), safe="/-_.~")
    creq = "\n".join([method, canon_path, canon_query, canon_headers, signed, payload_hash])
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, _sha256_hex(creq.encode())])
    sig = hmac.new(sigv4_signing_key(secret_key, date, region, service), sts.encode(), hashlib.sha256).hexdigest()
    out = {k: v for k, v in h.items() if k != "host"}
    out["Authorization"] = f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={signed}, Signature={sig}"
    return out


# ------------------------------------------------------------ HTTP helpers
def _open(url: str, headers: dict | None = None, timeout: float = 60.0):
    req = urllib.request.Request(url, headers=headers or {})
    try:
        return urllib.request.urlopen(req, timeout=timeout)
    except urllib.error.HTTPError as e:
        body = e.read()[:500].decode(errors="replace")
        raise RuntimeError(f"GET {url}: HTTP {e.code} {body}") from None


def _save(resp, dest: str) -> None:
    os.makedirs(os.path.dirname(dest) or ".", exist_ok=True)
    tmp = dest + ".part"
    with open(tmp, "wb") as f:
        while True:
            b = resp.read(_CHUNK)
            if not b:
                break
            f.write(b)
    os.replace(tmp, dest)


def _rel_key(key: str, prefix: str) -> str:
    """Object key -> path under out_dir (reference: strip the prefix once)."""
    return key.replace(prefix, "", 1).strip("/") if prefix else key.strip("/")


def _safe_join(root: str, rel: str) -> str:
    dest = os.path.normpath(os.path.join(root, rel))
    if not (dest == os.path.normpath(root) or dest.startswith(os.path.normpath(root) + os.sep)):
        raise RuntimeError(f"object key {rel!r} escapes the download directory")
    return dest


def _split_bucket(uri: str, prefix: str) -> tuple[str, str]:
    parts = uri[len(prefix):].split("/", 1)
    return parts[0], parts[1] if len(parts) > 1 else ""


class Storage:
    @staticmethod
    def download(uri: str, out_dir: str | None = None) -> str:
        if not uri:
            raise ValueError("empty model uri")
        if uri.startswith(_PVC_PREFIX):
            root = os.environ.get("SELDON_PVC_ROOT", "/mnt")
            uri = os.path.join(root, uri[len(_PVC_PREFIX):])
        is_local = uri.startswith(_LOCAL_PREFIX) or os.path.exists(uri)
        if out_dir is None:
            if is_local:
                return Storage._download_local(uri)
            out_dir = tempfile.mkdtemp(prefix="sca-model-")
        remote = uri.startswith((_GCS_PREFIX, _S3_PREFIX)) or re.search(_BLOB_RE, uri)
        mirror = os.environ.get("SELDON_STORAGE_MIRROR")
        if remote and mirror:
            p = urllib.parse.urlparse(uri)
            return Storage._download_local(os.path.join(mirror, p.netloc, p.path.lstrip("/")), out_dir)
        if uri.startswith(_GCS_PREFIX):
            Storage._download_gcs(uri, out_dir)
        elif uri.startswith(_S3_PREFIX):
            Storage._download_s3(uri, out_dir)
        elif re.search(_BLOB_RE, uri):
            Storage._download_blob(uri, out_dir)
        elif is_local:
            return Storage._download_local(uri, out_dir)
        else:
            raise RuntimeError(f"Cannot recognize storage type for {uri}\n'{_GCS_PREFIX}', '{_S3_PREFIX}', and "
                               f"'{_LOCAL_PREFIX}' are the current available storage type.")
        log.info("Successfully copied %s to %s", uri, out_dir)
        return out_dir

    # -------------------------------------------------------------- S3
    @staticmethod
    def _s3_endpoint() -> str:
        url = urllib.parse.urlparse(os.getenv("S3_ENDPOINT", ""))
        if url.scheme:
            return f"{url.scheme}://{url.netloc}"
        use_ssl = os.getenv("USE_SSL", "true").lower() not in ("0", "false", "no")
        host = url.path or "s3.amazonaws.com"
        return ("https://" if use_ssl else "http://") + host

    @staticmethod
    def _s3_get(url: str):
        ak, sk = os.getenv("AWS_ACCESS_KEY_ID", ""), os.getenv("AWS_SECRET_ACCESS_KEY", "")
        headers = {}
        if ak and sk:
            headers = sigv4_headers("GET", url, access_key=ak, secret_key=sk,
                                    region=os.getenv("AWS_REGION", "us-east-1"),
                                    session_token=os.getenv("AWS_SESSION_TOKEN") or None)
        return _open(url, headers)

    @staticmethod
    def _download_s3(uri: str, out_dir: str) -> None:
        bucket, prefix = _split_bucket(uri, _S3_PREFIX)
        base = f"{Storage._s3_endpoint()}/{_uri_encode(bucket)}"
        token, n = None, 0
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            body = Storage._s3_get(base + "?" + urllib.parse.urlencode(q, quote_via=urllib.parse.quote)).read()
            root = ET.fromstring(body)
            ns = root.tag[:root.tag.index("}") + 1] if root.tag.startswith("{") else ""
            for c in root.findall(f"{ns}Contents"):
                key = c.findtext(f"{ns}Key")
                rel = _rel_key(key, prefix)
                if not rel or key.endswith("/"):
                    continue
                url = f"{base}/{_uri_encode(key, safe='/-_.~')}"
                _save(Storage._s3_get(url), _safe_join(out_dir, rel))
                n += 1
            if root.findtext(f"{ns}IsTruncated") == "true":
                token = root.findtext(f"{ns}NextContinuationToken")
            else:
                break
        if n == 0:
            raise RuntimeError(f"no objects under {uri}")

    # -------------------------------------------------------------- GCS
    @staticmethod
    def _download_gcs(uri: str, out_dir: str) -> None:
        bucket, path = _split_bucket(uri, _GCS_PREFIX)
        host = os.getenv("STORAGE_EMULATOR_HOST", "https://storage.googleapis.com").rstrip("/")
        tok = os.getenv("GOOGLE_OAUTH_ACCESS_TOKEN")
        headers = {"Authorization": f"Bearer {tok}"} if tok else {}
        prefix = path if (not path or path.endswith("/")) else path + "/"
        page, n = None, 0
        while True:
            q = {"prefix": prefix}
            if page:
                q["pageToken"] = page
            url = f"{host}/storage/v1/b/{_uri_encode(bucket)}/o?" + urllib.parse.urlencode(q)
            listing = json.loads(_open(url, headers).read())
            for item in listing.get("items", []):
                name = item["name"]
                rel = _rel_key(name, path)
                if not rel or name.endswith("/"):
                    continue
                dl = f"{host}/storage/v1/b/{_uri_encode(bucket)}/o/{_uri_encode(name, safe='')}?alt=media"
                _save(_open(dl, headers), _safe_join(out_dir, rel))
                n += 1
            page = listing.get("nextPageToken")
            if not page:
                break
        if n == 0:
            raise RuntimeError(f"no objects under {uri}")

    # -------------------------------------------------------------- Azure
    @staticmethod
    def _download_blob(uri: str, out_dir: str) -> None:
        m = re.search(_BLOB_RE, uri)
        account, rest = m.group(1), m.group(2)
        container, prefix = (rest.split("/", 1) + [""])[:2]
        base = os.getenv("AZURE_BLOB_ENDPOINT", f"https://{account}.blob.core.windows.net").rstrip("/")
        sas = os.getenv("AZURE_STORAGE_SAS_TOKEN", "").lstrip("?")
        headers = {"x-ms-version": "2019-02-02"}
        marker, n = None, 0
        while True:
            q = {"restype": "container", "comp": "list", "prefix": prefix}
            if marker:
                q["marker"] = marker
            url = f"{base}/{container}?" + urllib.parse.urlencode(q) + ("&" + sas if sas else "")
            root = ET.fromstring(_open(url, headers).read())
            for b in root.iter("Blob"):
                name = b.findtext("Name")
                if not name or name.endswith("/"):
                    continue
                dl = f"{base}/{container}/{_uri_encode(name, safe='/-_.~')}" + ("?" + sas if sas else "")
                # Reference keeps the full blob name under out_dir.
                _save(_open(dl, headers), _safe_join(out_dir, name))
                n += 1
            marker = root.findtext("NextMarker")
            if not marker:
                break
        if n == 0:
            raise RuntimeError(f"no blobs under {uri}")

    # -------------------------------------------------------------- local
    @staticmethod
    def _download_local(uri: str, out_dir: str | None = None) -> str:
        local_path = uri.replace(_LOCAL_PREFIX, "", 1)
        if not os.path.exists(local_path):
            raise FileNotFoundError(f"Local path {uri} does not exist.")
        if out_dir is None:
            return local_path
        os.makedirs(out_dir, exist_ok=True)
        srcs = glob.glob(os.path.join(local_path, "*")) if os.path.isdir(local_path) else [local_path]
        for src in srcs:
            dest = os.path.join(out_dir, os.path.basename(src))
            if os.path.lexists(dest):
                if os.path.isdir(dest) and not os.path.islink(dest):
                    shutil.rmtree(dest)
                else:
                    os.remove(dest)
            os.symlink(os.path.abspath(src), dest)
        return out_dir

    @staticmethod
    def tempdir() -> str:
        return tempfile.mkdtemp(prefix="sca-model-")
