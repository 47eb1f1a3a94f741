"""rnnt_install_crash_report (include/rnnt_mi355x.h): a fatal signal prints every frame as shared object +
offset and the process still dies of that signal (the previous disposition takes over).  CPU only: the
fault is a NULL read from Python."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = """
import ctypes, sys
sys.path.insert(0, %r)
from rnnt_amd import _lib
assert _lib.lib().rnnt_install_crash_report() == 0
assert _lib.lib().rnnt_install_crash_report() == 0  # idempotent
ctypes.string_at(8)
""" % os.path.join(REPO, "rnnt-inference_amd")


def test_fault_names_objects():
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=120)
    assert r.returncode == -11, (r.returncode, r.stderr[-2000:])
    assert "rnnt crash report: signal 11 at address 0x8" in r.stderr, r.stderr[-2000:]
    frames = [ln for ln in r.stderr.splitlines() if ln.startswith("  #")]
    assert len(frames) >= 3 and any(".so" in ln and "+0x" in ln for ln in frames), r.stderr[-2000:]
