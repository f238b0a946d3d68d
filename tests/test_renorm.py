"""The renormalisation fast path (rtk::renormalized, csrc/rt_device.h) is
bit-identical to the reference's normalisation (vec3.h:26-29) -- checked on the
host by tests/native/renorm_check.cpp, which restates the device arithmetic
(length class from s = |a|^2, Markstein's corrected quotient with the correctly
rounded reciprocal) and compares it with sqrt + three IEEE divisions on
renormalised unit vectors, reflections, perturbed lengths and special
components, plus the quotient step alone over the exponent range."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_renormalized_matches_ieee_normalisation(tmp_path):
    exe = tmp_path / "renorm_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "renorm_check.cpp")], check=True)
    out = subprocess.run([str(exe), "3000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    w = out.stdout.split()
    assert w[0] == "checked" and int(w[1]) >= 15000000 and int(w[3]) > 3000000, out.stdout
    assert w[-1] == "0", out.stdout
