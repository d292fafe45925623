"""The frontend's client-side validation script (wwwroot/js/validation.js, the reference's
_ValidationScriptsPartial) evaluated by Node.js against the rule attributes the form renders."""
import json
import shutil
import subprocess
from pathlib import Path

import pytest

JS = Path(__file__).resolve().parents[1] / "aca_dotnet_workshop_amd" / "services" / "frontend" / "wwwroot" / "js" / "validation.js"

CASES = [  # (value, attributes, expected message)
    ("", {"data-val": "true", "data-val-required": "The Task Name field is required."}, "The Task Name field is required."),
    ("   ", {"data-val": "true", "data-val-required": "req"}, "req"),
    ("Buy milk", {"data-val": "true", "data-val-required": "req"}, ""),
    ("bob", {"data-val": "true", "data-val-required": "req", "data-val-email": "bad email"}, "bad email"),
    ("bob@x.com", {"data-val": "true", "data-val-required": "req", "data-val-email": "bad email"}, ""),
    ("2030-13-45", {"data-val": "true", "data-val-date": "bad date"}, "bad date"),
    ("2030-06-07", {"data-val": "true", "data-val-date": "bad date"}, ""),
    ("", {"data-val": "true", "data-val-email": "bad email"}, ""),  # optional + empty: valid
    ("", {"data-val-required": "req"}, ""),                          # no data-val: not validated
]


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_validation_rules_in_node():
    script = (f"const v = require({json.dumps(str(JS))});\n"
              f"const cases = {json.dumps(CASES)};\n"
              "console.log(JSON.stringify(cases.map(([val, attrs]) => "
              "v.check(val, n => (n in attrs ? attrs[n] : null)))));")
    out = subprocess.run(["node", "-e", script], capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stderr
    assert json.loads(out.stdout) == [c[2] for c in CASES]
