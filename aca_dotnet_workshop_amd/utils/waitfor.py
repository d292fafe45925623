"""Wait until an HTTP endpoint answers -- the walkthroughs' "the app has started" step.

    python -m aca_dotnet_workshop_amd.utils.waitfor http://127.0.0.1:7088/api/tasks [--timeout 30]

Exits 0 at the first HTTP response (any status unless ``--status`` is given), 1 on timeout.
HTTPS certificates are not verified (the environment CA is local).
"""
from __future__ import annotations

import argparse
import ssl
import sys
import time
import urllib.error
import urllib.request


def wait(url: str, timeout: float = 30.0, status: int | None = None) -> bool:
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        try:
            with urllib.request.urlopen(url, timeout=2, context=ctx) as r:
                code = r.status
        except urllib.error.HTTPError as e:
            code = e.code
        except (OSError, urllib.error.URLError):
            time.sleep(0.1)
            continue
        if status is None or code == status:
            return True
        time.sleep(0.1)
    return False


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="waitfor")
    ap.add_argument("url")
    ap.add_argument("--timeout", type=float, default=30.0)
    ap.add_argument("--status", type=int, default=None)
    a = ap.parse_args(argv)
    if wait(a.url, a.timeout, a.status):
        return 0
    print(f"waitfor: {a.url} did not answer within {a.timeout:.0f}s", file=sys.stderr)
    return 1


if __name__ == "__main__":
    sys.exit(main())
