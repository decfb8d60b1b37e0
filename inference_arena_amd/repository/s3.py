"""Minimal S3 / MinIO client for the model repository (no SDK dependency).

The reference distributes models through a MinIO bucket: ``MinIOModelRegistry``
waits for the server (tenacity, 10 tries, exponential 1-10 s), creates the
bucket, uploads ``<m>/1/model.onnx``, ``<m>/config.pbtxt`` and
``<m>/metadata.json`` skipping objects that already exist unless ``--force``
(infrastructure/minio/init_models.py:116-405, :167-183, :200-273), and init
containers ``fget_object`` the files into each service's model volume
(architectures/*/init_*_models.py).  The ``minio`` package is not available
here, so this module speaks the S3 REST protocol directly: AWS Signature V4
request signing (hashlib/hmac), path-style URLs (MinIO's default), and the
handful of calls the repository needs — HEAD/PUT bucket, PUT/GET/HEAD object,
ListObjectsV2.

Connection settings default to experiment.yaml ``infrastructure.minio`` and
can be overridden with the reference's env names (``MINIO_INTERNAL_ENDPOINT``,
``MINIO_ACCESS_KEY``, ``MINIO_SECRET_KEY``, ``MINIO_BUCKET``, ``MINIO_SECURE``).
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import hmac
import os
import time
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from pathlib import Path

EMPTY_SHA256 = hashlib.sha256(b"").hexdigest()


class S3Error(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"S3 error {status}: {message}")
        self.status = status


def _sha256(data: bytes) -> str:
    return hashlib.sha256(data).hexdigest()


def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode("utf-8"), hashlib.sha256).digest()


def _quote(s: str, safe: str = "-_.~") -> str:
    return urllib.parse.quote(s, safe=safe)


def sign_v4(method: str, host: str, path: str, query: dict[str, str], headers: dict[str, str], payload_hash: str,
            access_key: str, secret_key: str, region: str, amz_date: str, service: str = "s3") -> dict[str, str]:
    """Headers of a SigV4-signed request (``Authorization``, ``x-amz-date``, ``x-amz-content-sha256`` added).

    ``path`` is the URI-encoded absolute path, ``query`` the decoded query parameters."""
    date = amz_date[:8]
    hdrs = {k.lower(): " ".join(str(v).strip().split()) for k, v in headers.items()}
    hdrs["host"] = host
    hdrs["x-amz-date"] = amz_date
    hdrs["x-amz-content-sha256"] = payload_hash
    signed = sorted(hdrs)
    canonical_query = "&".join(f"{_quote(k)}={_quote(v)}" for k, v in sorted(query.items()))
    canonical = "\n".join([
        method,
        path,
        canonical_query,
        "".join(f"{k}:{hdrs[k]}\n" for k in signed),
        ";".join(signed),
        payload_hash,
    ])
    scope = f"{date}/{region}/{service}/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, _sha256(canonical.encode("utf-8"))])
    k = _hmac(("AWS4" + secret_key).encode("utf-8"), date)
    k = _hmac(k, region)
    k = _hmac(k, service)
    k = _hmac(k, "aws4_request")
    sig = hmac.new(k, to_sign.encode("utf-8"), hashlib.sha256).hexdigest()
    out = dict(headers)
    out["x-amz-date"] = amz_date
    out["x-amz-content-sha256"] = payload_hash
    out["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={';'.join(signed)}, "
                            f"Signature={sig}")
    return out


@dataclass
class ObjectInfo:
    key: str
    size: int
    etag: str = ""


class S3Client:
    def __init__(self, endpoint: str, access_key: str, secret_key: str, *, secure: bool = False,
                 region: str = "us-east-1", timeout: float = 30.0):
        self.host = endpoint.replace("http://", "").replace("https://", "").rstrip("/")
        self.scheme = "https" if secure or endpoint.startswith("https://") else "http"
        self.access_key, self.secret_key, self.region, self.timeout = access_key, secret_key, region, timeout

    @classmethod
    def from_config(cls, **overrides) -> "S3Client":
        """Endpoint/credentials from experiment.yaml ``infrastructure.minio`` + reference env overrides."""
        from ..config import get_minio_config

        try:
            cfg = dict(get_minio_config())
        except KeyError:
            cfg = {}
        endpoint = os.environ.get("MINIO_INTERNAL_ENDPOINT", cfg.get("endpoint", "127.0.0.1:9000"))
        access = os.environ.get("MINIO_ACCESS_KEY", cfg.get("access_key", "minioadmin"))
        secret = os.environ.get("MINIO_SECRET_KEY", cfg.get("secret_key", "minioadmin"))
        secure = os.environ.get("MINIO_SECURE", str(cfg.get("secure", False))).lower() in ("1", "true", "yes")
        kw = {"endpoint": endpoint, "access_key": access, "secret_key": secret, "secure": secure}
        kw.update({k: v for k, v in overrides.items() if v is not None})
        return cls(kw.pop("endpoint"), kw.pop("access_key"), kw.pop("secret_key"), **kw)

    # ------------------------------------------------------------ transport
    def _request(self, method: str, bucket: str, key: str = "", *, query: dict[str, str] | None = None,
                 body: bytes = b"", headers: dict[str, str] | None = None) -> tuple[int, dict, bytes]:
        path = "/" + _quote(bucket, safe="-_.~") + ("/" + _quote(key, safe="-_.~/") if key else "")
        query = query or {}
        amz_date = _dt.datetime.now(_dt.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
        hdrs = sign_v4(method, self.host, path, query, dict(headers or {}), _sha256(body), self.access_key,
                       self.secret_key, self.region, amz_date)
        url = f"{self.scheme}://{self.host}{path}"
        if query:
            url += "?" + "&".join(f"{_quote(k)}={_quote(v)}" for k, v in sorted(query.items()))
        req = urllib.request.Request(url, data=body if method in ("PUT", "POST") else None, method=method,
                                     headers=hdrs)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return r.status, dict(r.headers), r.read()
        except urllib.error.HTTPError as e:
            return e.code, dict(e.headers or {}), e.read() if method != "HEAD" else b""

    # ------------------------------------------------------------ buckets
    def bucket_exists(self, bucket: str) -> bool:
        st, _, body = self._request("HEAD", bucket)
        if st in (200, 301, 403):
            return st == 200
        if st == 404:
            return False
        raise S3Error(st, body.decode("utf-8", "replace"))

    def make_bucket(self, bucket: str) -> None:
        st, _, body = self._request("PUT", bucket)
        if st not in (200, 409):  # 409: BucketAlreadyOwnedByYou
            raise S3Error(st, body.decode("utf-8", "replace"))

    def ensure_bucket(self, bucket: str) -> bool:
        """Create the bucket if missing; True when it was created."""
        if self.bucket_exists(bucket):
            return False
        self.make_bucket(bucket)
        return True

    # ------------------------------------------------------------ objects
    def put_object(self, bucket: str, key: str, data: bytes, content_type: str = "application/octet-stream") -> str:
        st, h, body = self._request("PUT", bucket, key, body=data, headers={"Content-Type": content_type})
        if st != 200:
            raise S3Error(st, body.decode("utf-8", "replace"))
        return str({k.lower(): v for k, v in h.items()}.get("etag", "")).strip('"')

    def fput_object(self, bucket: str, key: str, path: str | Path) -> str:
        return self.put_object(bucket, key, Path(path).read_bytes())

    def get_object(self, bucket: str, key: str) -> bytes:
        st, _, body = self._request("GET", bucket, key)
        if st != 200:
            raise S3Error(st, f"{bucket}/{key}: {body[:200].decode('utf-8', 'replace')}")
        return body

    def fget_object(self, bucket: str, key: str, path: str | Path) -> Path:
        p = Path(path)
        p.parent.mkdir(parents=True, exist_ok=True)
        tmp = p.with_suffix(p.suffix + ".part")
        tmp.write_bytes(self.get_object(bucket, key))
        tmp.replace(p)
        return p

    def stat_object(self, bucket: str, key: str) -> ObjectInfo | None:
        st, h, _ = self._request("HEAD", bucket, key)
        if st == 404:
            return None
        if st != 200:
            raise S3Error(st, f"HEAD {bucket}/{key}")
        hl = {k.lower(): v for k, v in h.items()}
        return ObjectInfo(key, int(hl.get("content-length", 0)), str(hl.get("etag", "")).strip('"'))

    def list_objects(self, bucket: str, prefix: str = "") -> list[ObjectInfo]:
        out: list[ObjectInfo] = []
        token = None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            st, _, body = self._request("GET", bucket, query=q)
            if st != 200:
                raise S3Error(st, body.decode("utf-8", "replace"))
            root = ET.fromstring(body)
            ns = root.tag.split("}")[0] + "}" if root.tag.startswith("{") else ""
            for c in root.findall(f"{ns}Contents"):
                out.append(ObjectInfo(c.findtext(f"{ns}Key", ""), int(c.findtext(f"{ns}Size", "0")),
                                      c.findtext(f"{ns}ETag", "").strip('"')))
            if root.findtext(f"{ns}IsTruncated", "false") != "true":
                return out
            token = root.findtext(f"{ns}NextContinuationToken")

    # ------------------------------------------------------------ readiness
    def wait_ready(self, bucket: str | None = None, attempts: int = 10, min_wait: float = 1.0,
                   max_wait: float = 10.0, sleep=time.sleep) -> None:
        """Retry until the server answers (the reference's tenacity policy: 10 tries, exponential 1-10 s)."""
        delay = min_wait
        last: Exception | None = None
        for i in range(attempts):
            try:
                self.bucket_exists(bucket or "arena-readiness-probe")
                return
            except (OSError, S3Error, urllib.error.URLError) as e:
                last = e
                if i + 1 < attempts:
                    sleep(delay)
                    delay = min(max_wait, delay * 2)
        raise ConnectionError(f"S3 endpoint {self.host} not ready after {attempts} attempts: {last}")


# ---------------------------------------------------------------- repository <-> bucket
def upload_repository(root: str | Path, client: S3Client, bucket: str, *, force: bool = False) -> dict[str, str]:
    """Upload every file of a local model repository under the same keys (``<m>/config.pbtxt``,
    ``<m>/metadata.json``, ``<m>/<v>/model.*``, ``checksums.txt``).  Existing objects of the same size
    are skipped unless ``force`` (reference: init_models.py:232-271).  Returns key -> 'uploaded' | 'skipped'."""
    root = Path(root)
    client.ensure_bucket(bucket)
    done: dict[str, str] = {}
    for p in sorted(x for x in root.rglob("*") if x.is_file()):
        key = p.relative_to(root).as_posix()
        if not force:
            st = client.stat_object(bucket, key)
            if st is not None and st.size == p.stat().st_size:
                done[key] = "skipped"
                continue
        client.fput_object(bucket, key, p)
        done[key] = "uploaded"
    return done


def download_repository(client: S3Client, bucket: str, dst: str | Path, *, models: list[str] | None = None,
                        force: bool = False) -> list[Path]:
    """Fetch a repository (or the listed models' prefixes) into ``dst`` with the same layout
    (the init-container step, architectures/triton/init_triton_models.py:25-142)."""
    dst = Path(dst)
    got: list[Path] = []
    prefixes = [f"{m}/" for m in models] if models else [""]
    for pre in prefixes:
        for obj in client.list_objects(bucket, pre):
            out = dst / obj.key
            if not force and out.exists() and out.stat().st_size == obj.size:
                continue
            got.append(client.fget_object(bucket, obj.key, out))
    return got
