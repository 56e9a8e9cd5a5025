"""The folded symmetric squaring's step algorithm (csrc/sliced28.h fold_*, build knob EFL_SQR_FOLD=1,
off by default since it measured slower) simulated lane by lane on the CPU: squares and
products equal the CIOS result (x + U m) / R bit for bit, accumulators within 64 bits."""
import os
import subprocess
import sys

from conftest import ROOT


def test_folded_steps_equal_cios():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "fold_sim.py"), "--trials", "4"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.count("equal the CIOS result") == 2
