"""Race detection / memory safety for the native engines (SURVEY.md §5 "Race detection /
sanitizers": the reference has none).  A multi-threaded stress program
(``native/tests/stress.cpp``) is compiled twice -- ThreadSanitizer, and AddressSanitizer +
UndefinedBehaviorSanitizer -- and must run clean.  Host code only (no GPU sanitizers)."""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "aca_dotnet_workshop_amd" / "native" / "tests" / "stress.cpp"
CXX = os.environ.get("CXX", "g++")


def _build_and_run(tmp_path, flags, env_extra, args=("8", "1500")):
    if shutil.which(CXX) is None:
        pytest.skip("no C++ compiler")
    exe = tmp_path / "stress"
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, str(SRC), "-o", str(exe), "-lpthread",
           "-lssl", "-lcrypto"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, **env_extra)
    run = subprocess.run([str(exe), *args, str(tmp_path / "store.log")], capture_output=True, text=True, env=env,
                         timeout=600)
    out = run.stdout + run.stderr
    assert run.returncode == 0, out[-5000:]
    assert "ALL OK" in run.stdout
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out and "runtime error" not in out
    return run.stdout


def test_native_engines_threadsanitizer(tmp_path):
    out = _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert "broker ok" in out and "docstore ok" in out and "backing front ok" in out


def test_native_engines_address_ub_sanitizer(tmp_path):
    out = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                         {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert "broker ok" in out


def test_dataplane_under_address_sanitizer(tmp_path):
    """The native sidecar data plane (callbacks, weak replies, pooled connections, the HTTP/2 +
    HPACK gRPC front) built with ASan+UBSan serves the full parity suite without a memory error: the suite's native cases run
    against the instrumented binary and any report fails the run (the data plane aborts)."""
    if shutil.which(CXX) is None:
        pytest.skip("no C++ compiler")
    exe = tmp_path / "ttsidecar-dataplane-asan"
    src = ROOT / "aca_dotnet_workshop_amd" / "native" / "src" / "dataplane.cpp"
    r = subprocess.run([CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", str(src), "-o", str(exe), "-lssl", "-lcrypto"],
                       capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, TT_DATAPLANE_BIN=str(exe), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               PYTHONPATH=str(ROOT))
    run = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                          str(ROOT / "tests" / "test_dataplane.py"), str(ROOT / "tests" / "test_grpc_api.py"),
                          str(ROOT / "tests" / "test_grpc_h2_native.py"), "-k", "native"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = run.stdout + run.stderr
    assert run.returncode == 0, out[-5000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out


@pytest.mark.parametrize("flags,env", [
    (["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"}),
    (["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"}),
], ids=["tsan", "asan-ubsan"])
def test_app_host_under_sanitizers(tmp_path, flags, env):
    """The app-process native host (``apphost.hpp``): the submitting thread and the I/O thread
    exchange 20k server requests and 20k client requests over Unix and TCP sockets; clean under
    ThreadSanitizer and ASan+UBSan."""
    if shutil.which(CXX) is None:
        pytest.skip("no C++ compiler")
    src = ROOT / "aca_dotnet_workshop_amd" / "native" / "tests" / "apphost_stress.cpp"
    exe = tmp_path / "apphost_stress"
    r = subprocess.run([CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, str(src), "-o", str(exe),
                        "-lpthread", "-lssl", "-lcrypto"], capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    run = subprocess.run([str(exe), "20000", "64", str(tmp_path / "ah.sock")], capture_output=True, text=True,
                         env=dict(os.environ, **env), timeout=600)
    out = run.stdout + run.stderr
    assert run.returncode == 0 and "ALL OK" in run.stdout, out[-5000:]
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out and "runtime error" not in out


def test_pipelined_connections_under_address_sanitizer(tmp_path):
    """The pipelined client connections (``evhttp.hpp`` PipeConn) against an evhttp server that
    answers out of order from timers and now and then drops every connection: each answer
    reaches its own request, the requests caught on a dropped connection fail once, later ones
    get through on new connections -- clean under ASan+UBSan (``native/tests/pipe_stress.cpp``)."""
    if shutil.which(CXX) is None:
        pytest.skip("no C++ compiler")
    src = ROOT / "aca_dotnet_workshop_amd" / "native" / "tests" / "pipe_stress.cpp"
    exe = tmp_path / "pipe_stress"
    r = subprocess.run([CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", str(src), "-o", str(exe), "-lpthread", "-lssl", "-lcrypto"],
                       capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    run = subprocess.run([str(exe), "20000", "64", str(tmp_path / "ps.sock")], capture_output=True, text=True,
                         env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"), timeout=300)
    out = run.stdout + run.stderr
    assert run.returncode == 0 and "ALL OK" in run.stdout, out[-5000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
