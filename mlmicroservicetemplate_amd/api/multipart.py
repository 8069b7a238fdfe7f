"""In-house ``multipart/form-data`` parser (RFC 7578 / RFC 2046 §5.1).

The reference's ``POST /predict`` takes the upload through FastAPI's ``File(...)``
(reference ``src/server/main.py:119-120``), which needs python-multipart -- not installed in
this image, so FastAPI ``File`` routes cannot even be declared.  This module
parses the body itself.  It works on the complete body (bounded by ``MAX_UPLOAD_BYTES``) with
``bytes.find`` so the scan runs at C speed, and exposes the parts as Starlette ``UploadFile``
objects so model plugins written against the reference contract (``predict(image_file)``
reading ``image_file.file``, reference ``src/model/model.py:16-23``) work unchanged.
"""
from __future__ import annotations

import io
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple
from urllib.parse import unquote

from starlette.datastructures import Headers, UploadFile


class MultipartError(ValueError):
    """Malformed multipart body (mapped to HTTP 400)."""


@dataclass
class Part:
    name: str
    data: bytes
    filename: Optional[str] = None
    content_type: Optional[str] = None
    headers: Dict[str, str] = field(default_factory=dict)

    @property
    def is_file(self) -> bool:
        return self.filename is not None

    def text(self, encoding: str = "utf-8") -> str:
        return self.data.decode(encoding)

    def to_upload_file(self) -> UploadFile:
        raw = [(k.encode("latin-1"), v.encode("latin-1")) for k, v in self.headers.items()]
        return UploadFile(
            file=io.BytesIO(self.data),
            size=len(self.data),
            filename=self.filename,
            headers=Headers(raw=raw),
        )


def parse_options_header(value: str) -> Tuple[str, Dict[str, str]]:
    """``form-data; name="a"; filename="b.png"`` -> (``form-data``, {name: a, filename: b.png}).

    Handles quoted strings with backslash escapes, ``;`` inside quotes and RFC 5987
    ``filename*=UTF-8''...`` extended values (which win over the plain form)."""
    value = value or ""
    parts: List[str] = []
    cur: List[str] = []
    in_q = esc = False
    for ch in value:
        if esc:
            cur.append(ch)
            esc = False
        elif ch == "\\" and in_q:
            cur.append(ch)
            esc = True
        elif ch == '"':
            in_q = not in_q
            cur.append(ch)
        elif ch == ";" and not in_q:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    parts.append("".join(cur))
    main = parts[0].strip().lower()
    params: Dict[str, str] = {}
    extended: Dict[str, str] = {}
    for p in parts[1:]:
        if "=" not in p:
            continue
        k, v = p.split("=", 1)
        k = k.strip().lower()
        v = v.strip()
        if len(v) >= 2 and v[0] == v[-1] == '"':
            v = v[1:-1]
            out = []
            i = 0
            while i < len(v):
                if v[i] == "\\" and i + 1 < len(v):
                    out.append(v[i + 1])
                    i += 2
                else:
                    out.append(v[i])
                    i += 1
            v = "".join(out)
        if k.endswith("*"):
            # charset'lang'percent-encoded
            pieces = v.split("'", 2)
            if len(pieces) == 3:
                charset = pieces[0] or "utf-8"
                try:
                    v = unquote(pieces[2], encoding=charset, errors="replace")
                except LookupError:
                    v = unquote(pieces[2])
            extended[k[:-1]] = v
        else:
            params[k] = v
    params.update(extended)
    return main, params


def boundary_from_content_type(content_type: Optional[str]) -> str:
    main, params = parse_options_header(content_type or "")
    if main != "multipart/form-data":
        raise MultipartError(f"expected multipart/form-data, got {main or 'no content type'}")
    b = params.get("boundary")
    if not b:
        raise MultipartError("multipart boundary missing")
    if len(b) > 200:
        raise MultipartError("multipart boundary too long")
    return b


def _parse_headers(block: bytes) -> Dict[str, str]:
    headers: Dict[str, str] = {}
    last: Optional[str] = None
    for raw in block.split(b"\r\n"):
        if not raw:
            continue
        if raw[:1] in (b" ", b"\t") and last is not None:  # obsolete line folding
            headers[last] += " " + raw.strip().decode("latin-1")
            continue
        if b":" not in raw:
            raise MultipartError("malformed part header")
        k, v = raw.split(b":", 1)
        last = k.strip().decode("latin-1").lower()
        headers[last] = v.strip().decode("latin-1")
    return headers


def parse_multipart(body: bytes, content_type: str, max_parts: int = 1000) -> Dict[str, List[Part]]:
    """Parse a complete multipart/form-data body into ``{field name: [Part, ...]}``."""
    boundary = boundary_from_content_type(content_type).encode("latin-1")
    delim = b"--" + boundary
    out: Dict[str, List[Part]] = {}
    # first delimiter may be at offset 0 or after a preamble line
    pos = body.find(delim)
    if pos < 0:
        raise MultipartError("multipart boundary not found in body")
    if pos > 0 and body[pos - 2 : pos] != b"\r\n":
        # a preamble must end in CRLF before the delimiter
        raise MultipartError("malformed multipart preamble")
    pos += len(delim)
    nparts = 0
    sep = b"\r\n" + delim
    while True:
        # after a delimiter: either "--" (close) or transport padding + CRLF
        if body[pos : pos + 2] == b"--":
            return out
        eol = body.find(b"\r\n", pos)
        if eol < 0:
            raise MultipartError("truncated multipart body")
        if body[pos:eol].strip(b" \t"):
            raise MultipartError("garbage after multipart boundary")
        hstart = eol + 2
        hend = body.find(b"\r\n\r\n", hstart)
        if hend < 0:
            # a part with no headers at all: CRLF immediately
            if body[hstart : hstart + 2] == b"\r\n":
                hend = hstart - 2
            else:
                raise MultipartError("truncated part headers")
        headers = _parse_headers(body[hstart:hend]) if hend > hstart else {}
        dstart = hend + 4
        dend = body.find(sep, dstart)
        if dend < 0:
            raise MultipartError("closing boundary not found")
        disp, params = parse_options_header(headers.get("content-disposition", ""))
        if disp != "form-data" or "name" not in params:
            raise MultipartError("part without form-data name")
        part = Part(
            name=params["name"],
            data=body[dstart:dend],
            filename=params.get("filename"),
            content_type=headers.get("content-type"),
            headers=headers,
        )
        out.setdefault(part.name, []).append(part)
        nparts += 1
        if nparts > max_parts:
            raise MultipartError("too many multipart parts")
        pos = dend + len(sep)


def encode_multipart(fields: Dict[str, Tuple[Optional[str], bytes, Optional[str]]], boundary: str = "mlsamd-boundary-7f3a") -> Tuple[bytes, str]:
    """Encoder used by the load generator and tests: ``{name: (filename, data, content_type)}``."""
    chunks: List[bytes] = []
    for name, (filename, data, ctype) in fields.items():
        disp = f'form-data; name="{name}"'
        if filename is not None:
            disp += f'; filename="{filename}"'
        chunks.append(f"--{boundary}\r\nContent-Disposition: {disp}\r\n".encode("latin-1"))
        if ctype:
            chunks.append(f"Content-Type: {ctype}\r\n".encode("latin-1"))
        chunks.append(b"\r\n")
        chunks.append(data)
        chunks.append(b"\r\n")
    chunks.append(f"--{boundary}--\r\n".encode("latin-1"))
    return b"".join(chunks), f"multipart/form-data; boundary={boundary}"
