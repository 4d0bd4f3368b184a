"""The decimal -> float64 conversion of kernel K0 (kcp_amd/csrc/decfloat.h:
Clinger's exact path, else Eisel-Lemire) against glibc's correctly rounded
strtod -- the host decoder's conversion (json.cpp), i.e. strconv.ParseFloat's
results -- on millions of random decimals over the full float64 range.  The
header is host+device code; this compiles it for the host."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_decimal_to_double_matches_strtod(tmp_path):
    exe = str(tmp_path / "decfloat_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tools", "decfloat_check.cpp")], check=True, capture_output=True)
    for seed in ("1", "2"):
        r = subprocess.run([exe, "1500000", seed], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        n, accepted, bad = map(int, r.stdout.split())
        assert bad == 0 and accepted > 0.9 * n, r.stdout
