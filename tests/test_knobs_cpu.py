"""Every MLOP_* environment knob the code reads is documented in docs/KNOBS.md."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_knob_documented():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "knobs.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
