"""The native data plane's HTTP/2 + HPACK + gRPC framing (native/src/h2.hpp), at the wire level.

``test_grpc_api.py`` proves API parity through ``grpcio`` (C-core); these tests talk raw frames to
the same port to pin the protocol corners a real client may use and a unary server must get
right: Huffman-coded and dynamically indexed headers (RFC 7541 Appendix C vectors), header
blocks split over CONTINUATION frames, padded frames, PING, request bodies split across DATA
frames, responses larger than the client's flow-control window (WINDOW_UPDATE), and connection
errors (bad preface, oversized frame, invalid Huffman padding / EOS).  A second, independent
HTTP/2 stack -- Node.js's ``http2`` client (nghttp2, which Huffman-codes and indexes headers on
its own terms) -- must interoperate as well.
"""
import asyncio
import json
import shutil
import struct
import subprocess

import pytest

from aca_dotnet_workshop_amd.sdk import proto as P

from helpers import run
from test_sidecar import Harness, _inline
from aca_dotnet_workshop_amd.web import WebApp

COSMOS = {"url": "https://acct.documents.azure.com:443/", "masterKey": "k", "database": "db", "collection": "c"}
PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"

# RFC 7541 Appendix B code lengths (the canonical code is rebuilt from them, as h2.hpp does)
_HUFF_LEN = bytes.fromhex(
    "0d171c1c1c1c1c1c1c181e1c1c1e1c1c1c1c1c1c1c1c1e1c1c1c1c1c1c1c1c1c060a0a0c0d06080b0a0a080b0806060605"
    "05050606060606060607080f060c0a0d06070707070707070707070707070707070707070707070807080d130d0e060f05"
    "060506050606060507070606060506070605050607070707070f0b0e0d1c141614141616161716171717171718171818"
    "161718171717171516171617171816151416161717151716161815161717151516151716171714161616171616171a1a"
    "1413161716191a1a1a1b1b1a181913151a1b1b1a1b1815151a1a1c1b1b1b14181415161515171616191918181a171a1b"
    "1a1a1b1b1b1b1b1c1b1b1b1b1b1a1e")


def _huff_codes():
    order = sorted(range(257), key=lambda s: (_HUFF_LEN[s], s))
    codes, code, prev = {}, 0, _HUFF_LEN[order[0]]
    for k, s in enumerate(order):
        n = _HUFF_LEN[s]
        if k:
            code = (code + 1) << (n - prev)
        prev = n
        codes[s] = (code, n)
    return codes


CODES = _huff_codes()


def huff(data: bytes, pad_bits: str | None = None) -> bytes:
    bits = "".join(format(CODES[b][0], f"0{CODES[b][1]}b") for b in data)
    if pad_bits is None:
        pad_bits = "1" * (-len(bits) % 8)
    bits += pad_bits
    bits += "1" * (-len(bits) % 8)
    return int(bits, 2).to_bytes(len(bits) // 8, "big") if bits else b""


def test_huffman_code_matches_rfc7541_vectors():
    # RFC 7541 C.4.1 / C.4.2 / C.6.1
    assert huff(b"www.example.com").hex() == "f1e3c2e5f23a6ba0ab90f4ff"
    assert huff(b"no-cache").hex() == "a8eb10649cbf"
    assert huff(b"custom-key").hex() == "25a849e95ba97d7f"
    assert huff(b"custom-value").hex() == "25a849e95bb8e8b4bf"
    assert huff(b"302").hex() == "6402"
    assert huff(b"private").hex() == "aec3771a4b"
    assert huff(b"https://www.example.com").hex() == "9d29ad171863c78f0b97c8e9ae82ae43d3"


# ------------------------------------------------------------------ raw HTTP/2 client
def frame(ftype: int, flags: int, sid: int, payload: bytes) -> bytes:
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


def hp_int(prefix_bits: int, first: int, v: int) -> bytes:
    mask = (1 << prefix_bits) - 1
    if v < mask:
        return bytes([first | v])
    out = bytearray([first | mask])
    v -= mask
    while v >= 128:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)
    return bytes(out)


def hp_str(s: bytes, use_huff: bool) -> bytes:
    if use_huff:
        h = huff(s)
        return hp_int(7, 0x80, len(h)) + h
    return hp_int(7, 0, len(s)) + s


def lit(name: bytes, value: bytes, use_huff=True, index=False) -> bytes:
    """Literal with a new name: incremental indexing (0x40) or without indexing (0x00)."""
    return bytes([0x40 if index else 0x00]) + hp_str(name, use_huff) + hp_str(value, use_huff)


def request_headers(method_path: str, token: str | None = None, use_huff=True, index=False) -> bytes:
    b = bytes([0x83, 0x86])  # :method POST, :scheme http (static)
    b += bytes([0x44]) + hp_str(method_path.encode(), use_huff)  # :path, literal w/ indexing, name idx 4
    b += bytes([0x41]) + hp_str(b"127.0.0.1", use_huff)          # :authority
    b += bytes([0x5F]) + hp_str(b"application/grpc", use_huff)   # content-type (idx 31), indexed
    b += lit(b"te", b"trailers", use_huff, index)
    if token:
        b += lit(b"dapr-api-token", token.encode(), use_huff, index)
    return b


def grpc_msg(m) -> bytes:
    body = m.SerializeToString()
    return b"\x00" + struct.pack(">I", len(body)) + body


class RawH2:
    """Blocking-free asyncio HTTP/2 client speaking raw frames; decodes only what our server sends
    (literals without indexing + the static :status 200)."""

    def __init__(self, port: int):
        self.port = port

    async def __aenter__(self):
        self.r, self.w = await asyncio.open_connection("127.0.0.1", self.port)
        return self

    async def __aexit__(self, *exc):
        self.w.close()

    def send(self, data: bytes):
        self.w.write(data)

    async def read_frame(self, timeout=5.0):
        hdr = await asyncio.wait_for(self.r.readexactly(9), timeout)
        n = int.from_bytes(hdr[:3], "big")
        payload = await asyncio.wait_for(self.r.readexactly(n), timeout) if n else b""
        return hdr[3], hdr[4], int.from_bytes(hdr[5:9], "big") & 0x7FFFFFFF, payload

    async def handshake(self, settings: bytes = b""):
        self.send(PREFACE + frame(4, 0, 0, settings))

    async def response(self, sid: int, window_updates=False):
        """Collect one stream's response: (headers, data, trailers); auto-ACKs SETTINGS."""
        headers, data, trailers = None, b"", None
        while True:
            t, f, s, p = await self.read_frame()
            if t == 4 and not f & 1:
                self.send(frame(4, 1, 0, b""))
                continue
            if t == 7:
                raise AssertionError(f"GOAWAY {p!r}")
            if s != sid:
                continue
            if t == 1:
                hl = decode_literals(p)
                if headers is None:
                    headers = hl
                else:
                    trailers = hl
                if f & 1:
                    return headers, data, trailers
            elif t == 0:
                data += p
                if window_updates and p:
                    self.send(frame(8, 0, 0, struct.pack(">I", len(p))) + frame(8, 0, sid, struct.pack(">I", len(p))))
                if f & 1:
                    return headers, data, trailers
            elif t == 3:
                raise AssertionError(f"RST_STREAM {p!r}")


def decode_literals(block: bytes) -> dict:
    out, i = {}, 0

    def integer(prefix):
        nonlocal i
        mask = (1 << prefix) - 1
        v = block[i] & mask
        i += 1
        if v < mask:
            return v
        shift = 0
        while True:
            b = block[i]
            i += 1
            v += (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                return v

    def string():
        nonlocal i
        assert not block[i] & 0x80, "server never Huffman-codes"
        n = integer(7)
        s = block[i:i + n].decode()
        i += n
        return s
    static = {8: (":status", "200"), 31: ("content-type", None)}
    while i < len(block):
        b = block[i]
        if b == 0x88:
            out[":status"] = "200"
            i += 1
            continue
        assert b & 0xF0 == 0, f"unexpected representation {b:#x}"
        idx = integer(4)
        name = static[idx][0] if idx else string()
        out[name] = string()
    return out


def grpc_payload(data: bytes) -> bytes:
    assert data[0] == 0
    n = int.from_bytes(data[1:5], "big")
    assert len(data) == 5 + n
    return data[5:]


# ------------------------------------------------------------------ tests
def _harness():
    comps = [_inline("statestore", "state.azure.cosmosdb", COSMOS)]
    return Harness(WebApp("h2app"), comps, app_id="h2app", grpc_port=0, data_plane="native")


def _save(key, value: bytes):
    m = P.rt("SaveStateRequest")(store_name="statestore")
    m.states.add(key=key, value=value)
    return m


def test_native_h2_huffman_indexing_continuation_padding_ping():
    async def main():
        async with _harness() as h, RawH2(h.sc.bound_grpc_port) as c:
            await c.handshake()
            # 1) Huffman strings + incremental indexing; request body split over 3 DATA frames
            msg = grpc_msg(_save("hk1", b'{"a":1}'))
            c.send(frame(1, 0x4, 1, request_headers("/dapr.proto.runtime.v1.Dapr/SaveState", index=True)))
            c.send(frame(0, 0, 1, msg[:3]) + frame(0, 0, 1, msg[3:10]) + frame(0, 1, 1, msg[10:]))
            hd, data, tr = await c.response(1)
            assert hd[":status"] == "200" and tr["grpc-status"] == "0", (hd, tr)
            # 2) same headers again as indexed dynamic-table references (62..), header block split
            #    over HEADERS + CONTINUATION, padded HEADERS and padded DATA
            #    (table after request 1: 62 te, 63 content-type, 64 :authority, 65 :path SaveState)
            block = bytes([0x83, 0x86, 0x04]) + hp_str(b"/dapr.proto.runtime.v1.Dapr/GetState", True)
            block += bytes([0x80 | 64, 0x80 | 63, 0x80 | 62])
            get = P.rt("GetStateRequest")(store_name="statestore", key="hk1")
            pad = 5
            c.send(frame(1, 0x8, 3, bytes([pad]) + block[:3] + b"\0" * pad))
            c.send(frame(9, 0x4, 3, block[3:]))
            body = grpc_msg(get)
            c.send(frame(0, 0x8 | 0x1, 3, bytes([2]) + body + b"\0\0"))
            hd, data, tr = await c.response(3)
            assert tr["grpc-status"] == "0", tr
            resp = P.rt("GetStateResponse").FromString(grpc_payload(data))
            assert json.loads(resp.data) == {"a": 1} and resp.etag
            # 3) PING is answered with the same payload
            c.send(frame(6, 0, 0, b"12345678"))
            while True:
                t, f, s, p = await c.read_frame()
                if t == 6:
                    assert f == 1 and p == b"12345678"
                    break
            # 4) error status as a trailers-only response, message percent-encoded
            c.send(frame(1, 0x4, 5, request_headers("/dapr.proto.runtime.v1.Dapr/GetState")))
            c.send(frame(0, 1, 5, grpc_msg(P.rt("GetStateRequest")(store_name="no storeé", key="x"))))
            hd, data, tr = await c.response(5)
            assert tr is None and hd["grpc-status"] == "3" and "%C3%A9" in hd["grpc-message"], hd
            assert hd["dapr-http-status"] == "400"
            # 5) unknown method of the service (bridged to the control plane) -> UNIMPLEMENTED
            c.send(frame(1, 0x4, 7, request_headers("/dapr.proto.runtime.v1.Dapr/NoSuchRpc")))
            c.send(frame(0, 1, 7, b"\0\0\0\0\0"))
            hd, _, _ = await c.response(7)
            assert hd["grpc-status"] == "12", hd
    run(main())


def test_native_h2_flow_control_large_response():
    """A 300 KB value read back with a 1000-byte initial stream window: the server must wait for
    WINDOW_UPDATEs, split by the peer's max frame size, and still deliver every byte."""
    big = json.dumps({"blob": "x" * 300_000}).encode()

    async def main():
        async with _harness() as h, RawH2(h.sc.bound_grpc_port) as c:
            await c.handshake(struct.pack(">HI", 0x4, 1000))  # SETTINGS_INITIAL_WINDOW_SIZE = 1000
            # request larger than one frame: 20 DATA frames of <= 16 KB
            msg = grpc_msg(_save("big", big))
            c.send(frame(1, 0x4, 1, request_headers("/dapr.proto.runtime.v1.Dapr/SaveState")))
            for off in range(0, len(msg), 16384):
                part = msg[off:off + 16384]
                c.send(frame(0, 1 if off + 16384 >= len(msg) else 0, 1, part))
            hd, _, tr = await c.response(1, window_updates=True)
            assert tr["grpc-status"] == "0", (hd, tr)
            c.send(frame(1, 0x4, 3, request_headers("/dapr.proto.runtime.v1.Dapr/GetState")))
            c.send(frame(0, 1, 3, grpc_msg(P.rt("GetStateRequest")(store_name="statestore", key="big"))))
            hd, data, tr = await c.response(3, window_updates=True)
            assert tr["grpc-status"] == "0"
            assert json.loads(P.rt("GetStateResponse").FromString(grpc_payload(data)).data) == json.loads(big)
    run(main())


@pytest.mark.parametrize("case", ["bad-preface", "oversized-frame", "huffman-eos", "huffman-bad-padding",
                                  "continuation-interleaved"])
def test_native_h2_connection_errors(case):
    async def main():
        async with _harness() as h, RawH2(h.sc.bound_grpc_port) as c:
            if case == "bad-preface":
                c.send(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
                # not HTTP/2: closed without a reply (at most our own preface SETTINGS went out first)
                data = await asyncio.wait_for(c.r.read(), 5)
                assert data == b"" or (data[3] == 4 and b"HTTP/" not in data), data
                return
            await c.handshake()
            if case == "oversized-frame":
                c.send(frame(0, 0, 1, b"\0" * 20000))
                want = 6  # FRAME_SIZE_ERROR
            elif case == "huffman-eos":
                eos = "1" * 30
                bad = bytes([0x00]) + hp_int(7, 0x80, 4) + int(eos + "11", 2).to_bytes(4, "big") + hp_str(b"v", False)
                c.send(frame(1, 0x5, 1, bytes([0x83, 0x86, 0x84]) + bad))
                want = 9  # COMPRESSION_ERROR
            elif case == "huffman-bad-padding":
                bad = bytes([0x00]) + hp_str(b"a", False) + bytes([0x81]) + huff(b"0", pad_bits="000")
                c.send(frame(1, 0x5, 1, bytes([0x83, 0x86, 0x84]) + bad))
                want = 9
            else:  # HEADERS without END_HEADERS followed by another stream's frame
                c.send(frame(1, 0x0, 1, bytes([0x83])) + frame(1, 0x4, 3, bytes([0x83])))
                want = 1  # PROTOCOL_ERROR
            while True:
                t, f, s, p = await c.read_frame()
                if t == 7:
                    assert int.from_bytes(p[4:8], "big") == want, p
                    break
            assert await asyncio.wait_for(c.r.read(), 5) == b""  # connection closed after GOAWAY
    run(main())


NODE_CLIENT = r"""
const http2 = require('http2');
const [port, save, get] = process.argv.slice(2);
const c = http2.connect('http://127.0.0.1:' + port);
function call(path, hex) {
  return new Promise((resolve, reject) => {
    const req = c.request({':method': 'POST', ':path': path, 'content-type': 'application/grpc', 'te': 'trailers',
                           'user-agent': 'node-http2-interop/1.0', 'x-custom-metadata': 'some value to huffman-code'});
    const chunks = []; let trailers = null;
    req.on('data', d => chunks.push(d));
    req.on('trailers', t => { trailers = t; });
    req.on('end', () => resolve({data: Buffer.concat(chunks).toString('hex'), trailers}));
    req.on('error', reject);
    req.end(Buffer.from(hex, 'hex'));
  });
}
(async () => {
  const out = [];
  for (let i = 0; i < 3; i++) {  // repeated headers: nghttp2 indexes them dynamically
    out.push(await call('/dapr.proto.runtime.v1.Dapr/SaveState', save));
    out.push(await call('/dapr.proto.runtime.v1.Dapr/GetState', get));
  }
  console.log(JSON.stringify(out));
  c.close();
})().catch(e => { console.error(e); process.exit(1); });
"""


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_native_h2_interop_with_nodejs_http2(tmp_path):
    script = tmp_path / "client.js"
    script.write_text(NODE_CLIENT)
    save = grpc_msg(_save("nodekey", b'{"from":"node"}')).hex()
    get = grpc_msg(P.rt("GetStateRequest")(store_name="statestore", key="nodekey")).hex()

    async def main():
        async with _harness() as h:
            proc = await asyncio.create_subprocess_exec("node", str(script), str(h.sc.bound_grpc_port), save, get,
                                                        stdout=subprocess.PIPE, stderr=subprocess.PIPE)
            out, err = await asyncio.wait_for(proc.communicate(), 30)
            assert proc.returncode == 0, err.decode()
            res = json.loads(out)
            assert len(res) == 6
            for r in res:
                assert r["trailers"]["grpc-status"] == "0", r
            got = P.rt("GetStateResponse").FromString(grpc_payload(bytes.fromhex(res[1]["data"])))
            assert json.loads(got.data) == {"from": "node"}
    run(main())
