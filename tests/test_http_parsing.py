"""Chunked transfer decoding of the Python HTTP server/client (``web/server.py``
``_ChunkedDecoder``): incremental, size-capped, strict about malformed size lines."""
import pytest

from aca_dotnet_workshop_amd.web import server as srv


def feed_all(parts):
    d = srv._ChunkedDecoder()
    buf = bytearray()
    out = None
    for i, p in enumerate(parts):
        buf += p
        out = d.feed(buf)
        if out is not None:
            return out, bytes(buf) + b"".join(parts[i + 1:])
    return out, bytes(buf)


def test_decodes_across_arbitrary_splits():
    wire = b"3\r\nabc\r\n5;ext=1\r\nhello\r\n0\r\nX-T: 1\r\n\r\nNEXT"
    for cut in range(1, len(wire)):
        body, rest = feed_all([wire[:cut], wire[cut:]])
        assert body == b"abchello"
        assert rest == b"NEXT"
    body, rest = feed_all([bytes([c]) for c in wire])  # byte at a time: linear, not re-decoded
    assert body == b"abchello" and rest == b"NEXT"


@pytest.mark.parametrize("wire", [
    b"zz\r\nabc\r\n0\r\n\r\n",                    # not hex
    b"\r\n\r\n",                                   # no digits (must not read as the last chunk)
    b"FFFFFFFFFFFFFFFFF\r\n",                      # saturating size
    b"3\r\nabcXY0\r\n\r\n",                        # missing CRLF after chunk data
])
def test_rejects_malformed(wire):
    with pytest.raises(ValueError):
        feed_all([wire])


def test_body_cap(monkeypatch):
    monkeypatch.setattr(srv, "MAX_BODY_BYTES", 10)
    with pytest.raises(ValueError, match="too large"):
        feed_all([b"8\r\n12345678\r\n8\r\n"])
    body, _ = feed_all([b"8\r\n12345678\r\n2\r\n90\r\n0\r\n\r\n"])
    assert body == b"1234567890"
