"""ttloadgen --pause-after (bench.py WarmLoadgen): the warmup's steps, a wait for the go line,
then the timed steps on the same connections, with figures for the timed steps only."""
import http.server
import json
import os
import subprocess
import threading
import time

import pytest

from aca_dotnet_workshop_amd.native import build


class _Handler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    connections: list = []

    def setup(self):
        super().setup()
        _Handler.connections.append(self.client_address)

    def do_POST(self):
        self.rfile.read(int(self.headers.get("content-length", 0)))
        self.send_response(302)
        self.send_header("Location", "/Tasks/Index")
        self.send_header("Content-Length", "0")
        self.end_headers()

    def log_message(self, *a):
        pass


@pytest.fixture(scope="module")
def loadgen():
    return str(build.build_loadgen())


def test_pause_after_reuses_the_warmup_connections(loadgen, tmp_path):
    _Handler.connections = []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    bodies = tmp_path / "bodies.txt"
    bodies.write_text("a=1\nb=2\n")
    cmd = [loadgen, "--target", f"127.0.0.1:{srv.server_address[1]}", "--path", "/Tasks/Create", "--bodies",
           str(bodies), "--concurrency", "2", "--batch", "8", "--steps", "3", "--expect", "302",
           "--pause-after", "1"]
    p = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        warm = json.loads(p.stdout.readline())
        assert warm["requests"] == 8 and warm["errors"] == 0 and len(warm["steps_ms"]) == 1
        time.sleep(0.3)
        assert p.poll() is None, "it must wait for the go line"
        p.stdin.write("go\n")
        p.stdin.flush()
        out = p.stdout.read()
        assert p.wait(timeout=60) == 0
        timed = json.loads(out.strip().splitlines()[-1])
        assert timed["requests"] == 16 and timed["status_counts"] == {"302": 16}
        assert len(timed["steps_ms"]) == 2
        assert len(_Handler.connections) == 2, _Handler.connections  # no new connection after the pause
    finally:
        if p.poll() is None:
            p.kill()
        srv.shutdown()


def test_pause_after_stops_when_the_parent_goes_away(loadgen, tmp_path):
    _Handler.connections = []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    bodies = tmp_path / "bodies.txt"
    bodies.write_text("a=1\n")
    p = subprocess.Popen([loadgen, "--target", f"127.0.0.1:{srv.server_address[1]}", "--bodies", str(bodies),
                          "--batch", "4", "--steps", "5", "--expect", "302", "--pause-after", "2"],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        assert json.loads(p.stdout.readline())["requests"] == 8
        p.stdin.close()  # no go line ever comes
        assert p.wait(timeout=60) == 0
    finally:
        if p.poll() is None:
            p.kill()
        srv.shutdown()


def test_pause_after_refuses_several_generators(loadgen):
    r = subprocess.run([loadgen, "--target", "127.0.0.1:1", "--threads", "2", "--concurrency", "4", "--batch", "8",
                        "--pause-after", "1"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "--pause-after" in r.stderr
    assert os.path.exists(loadgen)
