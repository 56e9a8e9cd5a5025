"""The SOS squaring's step algorithm (csrc/sliced28.h sos_sqr: the square by columns into LDS, then
the reduction over the lane-sliced window) simulated lane by lane on the CPU: squares equal the CIOS
result (x^2 + U m) / R bit for bit, LDS words within 32 bits, accumulators within 64."""
import os
import subprocess
import sys

from conftest import ROOT


def test_sos_steps_equal_cios():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sos_sim.py"), "--trials", "4"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.count("equal the CIOS result") == 2
